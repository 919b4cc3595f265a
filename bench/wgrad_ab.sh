#!/bin/bash
# k_wgrad_pp A/B on the GPU box: new-kernel tests, the weight-gradient shape bench with the kernel on / off, and the
# ResNet-50 batch-256 step with it on / off.  usage: bash bench/wgrad_ab.sh TAG
tag=${1:-ab}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad or weight_grad" > gpurun_out/pytest_wgrad_$tag.log 2>&1 && \
timeout -k 10 300 python bench/wgrad_bench.py > gpurun_out/wgrad_pp_$tag.log 2>&1 && \
DCA_OPS_WGRAD_PP=0 timeout -k 10 300 python bench/wgrad_bench.py > gpurun_out/wgrad_old_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_pp_$tag.log 2>&1 && \
DCA_OPS_WGRAD_PP=0 timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_old_$tag.log 2>&1
