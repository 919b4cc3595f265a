#!/bin/bash
# masked identity gradient for layer 3 too: ops tests, then ResNet-50 same-box A/B against the committed tree
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_ops_r4af.log 2>&1 && \
bash bench/ab_r50.sh gpurun_out/r50_l3_ab_r4af.log .l3base .
