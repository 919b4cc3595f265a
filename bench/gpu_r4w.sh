#!/bin/bash
# round-4 final tier on the committed tree: GPU tests, smoke, headline bench
mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_r4w.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4w.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_r4w.log 2>&1
