#!/bin/bash
# BN pass tuning: ops tests, then ResNet-50 same-box A/B (DCA_OPS_BN_TUNE=0 / 1, interleaved), then the micro-benchmark
mkdir -p gpurun_out
out=gpurun_out/r50_bntune_r4t.log
: > $out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ops_r4t.log 2>&1 || exit 1
for rep in 1 2; do
  for tune in 0 1; do
    echo "== tune=$tune rep=$rep" >> $out
    DCA_OPS_BN_TUNE=$tune timeout -k 10 200 python bench/resnet50.py --steps 30 --warmup 5 2>/dev/null | grep metric >> $out || exit 1
  done
done
timeout -k 10 200 ./bench/micro/bn_micro > gpurun_out/bn_micro_r4t.log 2>&1
