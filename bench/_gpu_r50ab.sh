set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_b256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_b256_fp8.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_b256_2.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_b256_fp8_2.log 2>&1
rc=$?
for f in r50_b256 r50_b256_fp8 r50_b256_2 r50_b256_fp8_2; do tail -1 gpurun_out/$f.log | cut -c1-150; done
exit $rc
