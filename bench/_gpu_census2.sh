set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 --fp8 > gpurun_out/census256_fp8.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_b256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_b256_fp8.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_ops.log
grep "conv-fwd" gpurun_out/census256_fp8.log | cut -c1-140; tail -1 gpurun_out/census256_fp8.log
for f in r50_b256 r50_b256_fp8; do tail -1 gpurun_out/$f.log | cut -c60-110; done
exit $rc
