set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_glds.log 2>&1 &&
DCA_OPS_GLDS_CONV=0 timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_noglds.log 2>&1 &&
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ops.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 8 --warmup 3 --path ops > gpurun_out/r50_b256.log 2>&1
rc=$?
paste -d' ' <(grep -v amdgpu gpurun_out/gemm_glds.log | cut -c1-80) <(grep -v amdgpu gpurun_out/gemm_noglds.log | cut -c30-60) | grep conv
tail -1 gpurun_out/pytest_ops.log; tail -1 gpurun_out/r50_b256.log | cut -c1-150
exit $rc
