set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_bn -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_bn.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
tail -1 gpurun_out/pytest_ops.log; tail -1 gpurun_out/r50.log | cut -c60-140
exit $rc
