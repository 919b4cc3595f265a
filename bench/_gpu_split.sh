# split-mode (two-phase persistent step) checks: numerics at ws=1, 2-rank DDP semantics (split is the ws>1
# default), and the ws=1 cost of the split
set -o pipefail
DCA_PK_SPLIT=1 timeout -k 10 300 python bench/engine_diag.py --batches 32,16 --persistent 1 > gpurun_out/diag_split.log 2>&1 &&
timeout -k 10 600 python -m pytest tests/test_ddp_engine_gpu.py -x -q > gpurun_out/pytest_ddp_split.log 2>&1 &&
DCA_PK_SPLIT=1 timeout -k 10 200 python bench.py --steps 500 --warmup 50 > gpurun_out/bench_split.log 2>&1
rc=$?
grep -E "summary|FAILED" gpurun_out/diag_split.log | cut -c1-300
tail -3 gpurun_out/pytest_ddp_split.log
tail -1 gpurun_out/bench_split.log | cut -c1-200
exit $rc
