#!/bin/bash
# ResNet-50 bench + kernel-trace profile after the BN tuning
mkdir -p gpurun_out
timeout -k 10 300 python bench/resnet50.py --steps 30 --warmup 5 > gpurun_out/r50_r4u.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_r4u -o r50 -- python3 bench/resnet50.py --steps 5 --warmup 2 > gpurun_out/prof_r50_r4u.log 2>&1
