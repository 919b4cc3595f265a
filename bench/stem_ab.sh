#!/bin/bash
# space-to-depth stem A/B + the sliced-engine check: stem / ops GPU tests, engine tests + bench, ResNet-50 with the
# s2d stem on / off / on.  usage: bash bench/stem_ab.sh TAG
tag=${1:-stem}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_stem_s2d.py \
  tests/test_ops_gpu.py > gpurun_out/pytest_ops_$tag.log 2>&1 && \
bash bench/engine_check.sh $tag && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_s2d_$tag.log 2>&1 && \
DCA_OPS_STEM_S2D=0 timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_nos2d_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_s2d2_$tag.log 2>&1
