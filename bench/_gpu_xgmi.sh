# xGMI one-shot all-reduce: multi-rank-on-one-GPU protocol tests, DDP semantics tests, 1-GPU bench unchanged.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_engine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_xgmi.log 2>&1 &&
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/pytest_xgmi.log | head -30
tail -1 gpurun_out/bench.log | cut -c1-250
exit $rc
