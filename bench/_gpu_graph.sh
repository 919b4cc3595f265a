set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 3 --batch 64 > gpurun_out/r50_64.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 3 --batch 64 --graph 1 > gpurun_out/r50_64g.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 --graph 1 > gpurun_out/r50_256g.log 2>&1 &&
timeout -k 10 300 python bench/resnet50.py --steps 10 --warmup 3 > gpurun_out/r50_256.log 2>&1
rc=$?
for f in r50_64 r50_64g r50_256g r50_256; do echo -n "$f "; tail -1 gpurun_out/$f.log | cut -c60-160; done
exit $rc
