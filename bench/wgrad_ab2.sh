#!/bin/bash
# after the shape-rule fix: wgrad tests, shape bench (rule), ResNet-50 A/B, then a kernel-trace profile of the step
tag=${1:-ab2}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py \
  -k "wgrad or weight_grad" > gpurun_out/pytest_wgrad_$tag.log 2>&1 && \
timeout -k 10 300 python bench/wgrad_bench.py > gpurun_out/wgrad_rule_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_pp_$tag.log 2>&1 && \
DCA_OPS_WGRAD_PP=0 timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_old_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_pp2_$tag.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_$tag -o r50 -- python3 bench/resnet50.py --steps 5 --warmup 2 > gpurun_out/prof_r50_$tag.log 2>&1
