# ops-layer kernel unit tests on the MI355X (one pytest process, time-boxed)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/pytest_ops.log | head -60
exit $rc
