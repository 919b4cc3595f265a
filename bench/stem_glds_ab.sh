#!/bin/bash
# the space-to-depth stem conv (C = 16) on the glds kernel with per-lane tap decode (DCA_OPS_GLDS_CONV_ANY=1) vs the
# register-staged k_gemm: stem tests under the flag, then ResNet-50 A/B on one box
tag=${1:-sg}
mkdir -p gpurun_out
DCA_OPS_GLDS_CONV_ANY=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread \
  tests/test_stem_s2d.py > gpurun_out/pytest_stem_glds_$tag.log 2>&1 && \
DCA_OPS_GLDS_CONV_ANY=1 timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_glds_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_reg_$tag.log 2>&1 && \
DCA_OPS_GLDS_CONV_ANY=1 timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_glds2_$tag.log 2>&1
