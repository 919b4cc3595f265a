#!/bin/bash
# kernel-trace profile of the final ResNet-50 step (batch 256)
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_r4aa -o r50 -- python3 bench/resnet50.py --steps 5 --warmup 2 > gpurun_out/prof_r50_r4aa.log 2>&1
