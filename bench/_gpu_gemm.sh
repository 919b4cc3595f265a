set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 --path ops > gpurun_out/r50_ops.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_ops.log
grep shape gpurun_out/gemm_bench.log
tail -1 gpurun_out/r50_ops.log | cut -c1-160
exit $rc
