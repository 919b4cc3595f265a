#!/bin/bash
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ops_r4k.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_r4k.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_r4k -o r50 -- python3 bench/resnet50.py --steps 5 --warmup 2 > gpurun_out/prof_r50_r4k.log 2>&1
