set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_glds.log 2>&1 &&
DCA_OPS_GLDS=0 timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_noglds.log 2>&1
rc=$?
paste -d' ' <(grep -v amdgpu gpurun_out/gemm_glds.log | cut -c1-80) <(grep -v amdgpu gpurun_out/gemm_noglds.log | cut -c30-60)
exit $rc
