# Rehearse the driver's multi-GPU bench command with 4 and 8 ranks sharing GPU 0 (gloo PG, xGMI IPC all-reduce path)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python bench.py --steps 300 --warmup 30 > gpurun_out/bench_n1.log 2>&1 &&
DCA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 4 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 4 --steps 200 --warmup 20 > gpurun_out/bench_share4.log 2>&1 &&
DCA_BENCH_SHARE_GPU=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 8 --steps 200 --warmup 20 > gpurun_out/bench_share8.log 2>&1
rc=$?
for f in bench_n1 bench_share4 bench_share8; do echo "== $f"; grep metric gpurun_out/$f.log | cut -c80-330; done
exit $rc
