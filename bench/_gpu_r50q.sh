set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops > gpurun_out/r50_ops.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r50 -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 5 --warmup 2 --path ops > $GRAFT_REPO_ROOT/gpurun_out/prof_r50.log 2>&1)
rc=$?
tail -2 gpurun_out/pytest_ops.log
tail -1 gpurun_out/r50_ops.log | cut -c1-160
exit $rc
