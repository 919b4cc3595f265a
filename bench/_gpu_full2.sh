# Full GPU tier + smoke + bench + ResNet-50 rocprof summary
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_r50e -o run -- python3 $GRAFT_REPO_ROOT/bench/resnet50.py --steps 4 --warmup 2 > $GRAFT_REPO_ROOT/gpurun_out/prof_r50e.log 2>&1
rc=$?
cd $GRAFT_REPO_ROOT
grep -E "passed|failed" gpurun_out/pytest_gpu.log | tail -3
grep -E "FAIL" gpurun_out/pytest_gpu.log | head
tail -1 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log | cut -c1-200
exit $rc
