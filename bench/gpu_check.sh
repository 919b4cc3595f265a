#!/bin/bash
# GPU-box check of the tree: default bench (bf16 + fp32) then the full GPU test tier, each under its own limit.
# usage (from the repo root, on the box): bash bench/gpu_check.sh TAG
tag=${1:-check}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1 && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_gpu_$tag.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1
