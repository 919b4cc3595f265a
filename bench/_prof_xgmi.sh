# 2 ranks sharing one MI355X (rehearsal of the multi-GPU bench): throughput and the xGMI all-reduce kernel's cost
set -o pipefail
mkdir -p gpurun_out
export DCA_BENCH_SHARE_GPU=1 DCA_XGMI_TIMEOUT_S=60
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29677 bench.py --gpus 2 --steps 300 --warmup 30 > gpurun_out/bench_share2.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29678 bench.py --gpus 2 --steps 300 --warmup 30 --allreduce xgmi --engine multikernel > gpurun_out/bench_share2_mk.log 2>&1 &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_xgmi -o run -- python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29679 $GRAFT_REPO_ROOT/bench.py --gpus 2 --steps 200 --warmup 20 > $GRAFT_REPO_ROOT/gpurun_out/prof_xgmi.log 2>&1)
rc=$?
grep metric gpurun_out/bench_share2.log | cut -c1-220
grep metric gpurun_out/bench_share2_mk.log | cut -c1-220
ls gpurun_out/prof_xgmi | head
exit $rc
