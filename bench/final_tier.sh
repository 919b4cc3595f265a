#!/bin/bash
# final tree on the GPU box: the full GPU tier, smoke, bench, and a kernel-trace profile of the ResNet-50 step
tag=${1:-final}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu_$tag.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_$tag.log 2>&1 && \
timeout -k 10 300 python bench/resnet50.py --steps 20 --warmup 5 > gpurun_out/r50_$tag.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r50_$tag -o r50 -- python3 bench/resnet50.py --steps 5 --warmup 2 > gpurun_out/prof_r50_$tag.log 2>&1
