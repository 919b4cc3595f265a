#!/bin/bash
# xGMI comm rehearsals (ws 2..8, measured crossover), headline bench, ResNet-50 bf16 vs --fp8 on one box
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_xgmi_comm_gpu.py -x -v -s --timeout 300 --timeout-method thread \
  > gpurun_out/pytest_xgmi_r4l.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r4l.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 30 --warmup 5 > gpurun_out/r50_bf16_r4l.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 30 --warmup 5 --fp8 > gpurun_out/r50_fp8_r4l.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 30 --warmup 5 > gpurun_out/r50_bf16b_r4l.log 2>&1
