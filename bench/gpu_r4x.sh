#!/bin/bash
# ResNet-50 after the BN tuning: batch 512 / 1024 (288 GB per GPU) and eval-mode throughput
mkdir -p gpurun_out
out=gpurun_out/r50_batch_infer_r4x.log
: > $out
for b in 512 1024; do
  echo "== batch $b" >> $out
  timeout -k 10 300 python bench/resnet50.py --batch $b --steps 10 --warmup 3 2>/dev/null | grep metric >> $out || exit 1
done
echo "== infer batch 256" >> $out
timeout -k 10 300 python bench/resnet50.py --infer --steps 30 --warmup 5 2>/dev/null | grep metric >> $out
