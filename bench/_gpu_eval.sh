# ops-layer inference path + PPE ROI model on the ops kernels
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_ppe.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_eval.log 2>&1
rc=$?
grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/pytest_eval.log | tail -40
exit $rc
