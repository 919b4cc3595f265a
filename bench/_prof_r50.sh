# ResNet-50 ops path at batch 256: GEMM census + rocprofv3 kernel stats
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r50b -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r50b.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
head -40 gpurun_out/census256.log; tail -1 gpurun_out/census256.log
find gpurun_out/prof_r50b -name "*stats*"
exit $rc
