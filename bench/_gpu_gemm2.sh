# ops tests + bs256 GEMM census + ResNet-50 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --path ops > gpurun_out/r50_b256.log 2>&1
rc=$?
tail -2 gpurun_out/pytest_ops.log
head -16 gpurun_out/census256.log | cut -c1-140; tail -1 gpurun_out/census256.log
tail -1 gpurun_out/r50_b256.log | cut -c1-170
exit $rc
