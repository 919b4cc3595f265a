# Generic xGMI communicator: multi-rank-on-one-GPU protocol tests (exact sums, FlatBucketDDP on the xGMI path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_xgmi_comm_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_comm.log 2>&1
rc=$?
tail -25 gpurun_out/pytest_comm.log
exit $rc
