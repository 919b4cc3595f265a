set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 8 --warmup 3 --path ops > gpurun_out/r50_b256.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 8 --warmup 3 --path ops --fp8 > gpurun_out/r50_b256_fp8.log 2>&1
rc=$?
for f in r50_b256 r50_b256_fp8; do tail -1 gpurun_out/$f.log | cut -c1-170; done
exit $rc
