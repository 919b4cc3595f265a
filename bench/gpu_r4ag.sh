#!/bin/bash
# final tier after the masked identity gradient: all GPU tests, smoke, headline bench, ResNet-50 at batch 256 / 512
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4ag.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4ag.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_r4ag.log 2>&1 && \
timeout -k 10 200 python bench/resnet50.py --steps 30 --warmup 5 > gpurun_out/r50_256_r4ag.log 2>&1 && \
timeout -k 10 200 python bench/resnet50.py --batch 512 --steps 15 --warmup 3 > gpurun_out/r50_512_r4ag.log 2>&1
