# GPU test tier in one gpurun call (one pytest process; every GPU step time-boxed, chained with &&)
set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1
rc=$?
tail -30 gpurun_out/pytest_gpu.log
exit $rc
