#!/bin/bash
# smoke, headline bench, ResNet-50 bench, and kernel-trace profiles of both steps on the current tree
mkdir -p gpurun_out
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r4p.log 2>&1 && \
timeout -k 10 300 python bench.py > gpurun_out/bench_r4p.log 2>&1 && \
timeout -k 10 300 python bench.py --steps 300 --warmup 30 > gpurun_out/bench300_r4p.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_pks_r4p -o pks -- python3 bench.py --steps 200 --warmup 20 --no-fp32 > gpurun_out/prof_pks_r4p.log 2>&1
