set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py > gpurun_out/gemm_bench.log 2>&1
rc=$?
grep shape gpurun_out/gemm_bench.log
exit $rc
