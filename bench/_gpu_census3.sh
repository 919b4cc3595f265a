set -o pipefail
mkdir -p gpurun_out
DCA_OPS_GLDS_CONV=1 timeout -k 10 300 python bench/r50_gemm_census.py --batch 256 > gpurun_out/census256_gc.log 2>&1 &&
DCA_OPS_GLDS_CONV=1 timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_gc.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50.log 2>&1
rc=$?
grep "conv-fwd" gpurun_out/census256_gc.log | cut -c1-140; tail -1 gpurun_out/census256_gc.log
for f in r50_gc r50; do echo -n "$f "; tail -1 gpurun_out/$f.log | cut -c60-110; done
exit $rc
