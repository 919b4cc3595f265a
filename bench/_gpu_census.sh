# ResNet-50 ops path: per-shape GEMM census (bs 64) + batch-size sweep
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/r50_gemm_census.py --batch 64 > gpurun_out/census64.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --path ops --batch 128 > gpurun_out/r50_b128.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --path ops --batch 256 > gpurun_out/r50_b256.log 2>&1
rc=$?
head -30 gpurun_out/census64.log; tail -1 gpurun_out/census64.log
for f in r50_b128 r50_b256; do tail -1 gpurun_out/$f.log | cut -c1-200; done
exit $rc
