set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_fp8.log 2>&1
rc=$?
tail -3 gpurun_out/pytest_ops.log; tail -1 gpurun_out/census256.log
for f in r50 r50_fp8; do echo -n "$f "; tail -1 gpurun_out/$f.log | cut -c60-140; done
exit $rc
