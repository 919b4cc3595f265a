#!/bin/bash
# residual link + explicit-FMA BN backward: diagnostic, ops tests, ResNet-50 same-box A/B (link off / on)
mkdir -p gpurun_out
timeout -k 10 300 python bench/diag_reslink.py > gpurun_out/diag_reslink_r4ac.log 2>&1 && \
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ops_r4ac.log 2>&1 || exit 1
out=gpurun_out/r50_reslink_ab_r4ac.log
: > $out
for rep in 1 2; do
  for rl in 0 1; do
    echo "== res_link=$rl rep=$rep" >> $out
    DCA_OPS_RES_LINK=$rl timeout -k 10 200 python bench/resnet50.py --steps 30 --warmup 5 2>/dev/null | grep metric >> $out || exit 1
  done
done
