# xGMI all-reduce protocol latency with 2 and 4 ranks sharing one MI355X (each step prints directly)
set -o pipefail
mkdir -p gpurun_out
export DCA_BENCH_SHARE_GPU=1 DCA_XGMI_TIMEOUT_S=60
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29681 bench/xgmi_allreduce_bench.py 2>&1 | tee gpurun_out/xgmi_bench2.log &&
timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29682 bench/xgmi_allreduce_bench.py 2>&1 | tee gpurun_out/xgmi_bench4.log
