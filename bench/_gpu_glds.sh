# glds GEMM: tests, GEMM microbench with/without glds, ResNet-50 bench
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_glds.log 2>&1 &&
DCA_OPS_GLDS=0 timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_noglds.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --path ops > gpurun_out/r50_b256.log 2>&1
rc=$?
tail -1 gpurun_out/pytest_ops.log
grep -v amdgpu gpurun_out/gemm_glds.log | cut -c1-100; echo ---; grep -v amdgpu gpurun_out/gemm_noglds.log | cut -c1-100
tail -1 gpurun_out/r50_b256.log | cut -c1-170
exit $rc
