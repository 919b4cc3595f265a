#!/bin/bash
# end-of-session check of the tree on the GPU box: engine tests, bench (bf16 + fp32) twice, the full GPU tier, smoke,
# and a kernel-trace profile of the headline bench.  usage: bash bench/final_check.sh TAG
tag=${1:-final}
mkdir -p gpurun_out
bash bench/engine_check.sh $tag && \
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/pytest_gpu_$tag.log 2>&1 && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$tag.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bench_$tag -o bench -- python3 bench.py --steps 200 --warmup 20 --no-fp32 > gpurun_out/prof_bench_$tag.log 2>&1
