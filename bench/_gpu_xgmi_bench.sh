# xGMI all-reduce: multi-rank protocol tests, then latency with 2 ranks sharing one MI355X
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ddp_engine_gpu.py -x -q --timeout 300 --timeout-method thread 2>&1 | tee gpurun_out/pytest_xgmi.log &&
DCA_BENCH_SHARE_GPU=1 DCA_XGMI_TIMEOUT_S=60 timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29681 bench/xgmi_allreduce_bench.py 2>&1 | tee gpurun_out/xgmi_bench2.log
