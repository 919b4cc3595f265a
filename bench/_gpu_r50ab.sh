set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_b256.log 2>&1 &&
DCA_FP8_MIN_CIN=256 timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_fp8_256.log 2>&1 &&
DCA_FP8_MIN_CIN=512 timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_fp8_512.log 2>&1 &&
DCA_FP8_MIN_CIN=1024 timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_fp8_1024.log 2>&1 &&
DCA_FP8_MIN_CIN=99999 timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --fp8 > gpurun_out/r50_fp8_none.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_b256_2.log 2>&1
rc=$?
for f in r50_b256 r50_fp8_256 r50_fp8_512 r50_fp8_1024 r50_fp8_none r50_b256_2; do echo -n "$f "; tail -1 gpurun_out/$f.log | cut -c60-110; done
exit $rc
