# rocprofv3 kernel stats of the ResNet-50 ops path (bf16)
set -o pipefail
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r50 -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 5 --warmup 2 --path ops > $GRAFT_REPO_ROOT/gpurun_out/prof_r50.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -1 gpurun_out/prof_r50.log | cut -c1-200
exit $rc
