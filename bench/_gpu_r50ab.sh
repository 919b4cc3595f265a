set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 6 --warmup 2 --batch 512 > gpurun_out/r50_512.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 8 --warmup 2 --batch 384 > gpurun_out/r50_384.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 12 --warmup 3 --batch 128 > gpurun_out/r50_128.log 2>&1
rc=$?
for f in r50_512 r50_384 r50_128; do echo -n "$f "; tail -1 gpurun_out/$f.log | cut -c60-160; done
exit $rc
