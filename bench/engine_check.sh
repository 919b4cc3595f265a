#!/bin/bash
# sliced-engine change check on the GPU box: engine / DDP GPU tests, then bench.py twice (bf16 + fp32 each)
tag=${1:-eng}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py \
  tests/test_ddp_engine_gpu.py > gpurun_out/pytest_engine_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_${tag}_1.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_${tag}_2.log 2>&1
