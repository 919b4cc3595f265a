set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
DCA_OPS_GLDS_CONV_ANY=1 timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or resnet" > gpurun_out/pytest_any.log 2>&1 &&
timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census_a.log 2>&1 &&
DCA_OPS_GLDS_CONV_ANY=1 timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census_b.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_ops.log; tail -1 gpurun_out/pytest_any.log
grep "392\|3211264" gpurun_out/census_a.log | cut -c1-120; grep "392\|3211264" gpurun_out/census_b.log | cut -c1-120
tail -1 gpurun_out/census_a.log; tail -1 gpurun_out/census_b.log
tail -1 gpurun_out/r50.log | cut -c60-140
exit $rc
