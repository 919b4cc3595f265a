#!/bin/bash
# 1024-thread BN finalize: BN op tests, then ResNet-50 same-box A/B against the committed tree (.finbase)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread -k "batch_norm or resnet or conv_bn" > gpurun_out/pytest_ops_r4v.log 2>&1 && \
bash bench/ab_r50.sh gpurun_out/r50_fin_ab_r4v.log .finbase .
