#!/bin/bash
# masked identity gradient: ops tests, then ResNet-50 same-box A/B (DCA_OPS_MASKED_JOIN=0 / 1, interleaved)
mkdir -p gpurun_out
out=gpurun_out/r50_maskjoin_ab_r4y.log
: > $out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ops_r4y.log 2>&1 || exit 1
for rep in 1 2; do
  for mj in 0 1; do
    echo "== masked_join=$mj rep=$rep" >> $out
    DCA_OPS_MASKED_JOIN=$mj timeout -k 10 200 python bench/resnet50.py --steps 30 --warmup 5 2>/dev/null | grep metric >> $out || exit 1
  done
done
