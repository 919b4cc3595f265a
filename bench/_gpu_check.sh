# Re-entry check in one gpurun call: GPU test tier, smoke, 1-GPU bench, rocprofv3 kernel stats.
# Every GPU step is time-boxed and chained with && so nothing else starts on the GPU after a failure.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof.log 2>&1)
rc=$?
tail -5 gpurun_out/pytest_gpu.log
tail -2 gpurun_out/smoke.log
tail -1 gpurun_out/bench.log | cut -c1-300
exit $rc
