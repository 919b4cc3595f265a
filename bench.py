"""Headline benchmark: whole-node images/sec of NetResDeep CIFAR-10 DDP training on MI355X.

Metric/config from BASELINE.json: "images/sec (whole node) CIFAR-10 ResNet at 1/2/4/8 MI355X; scaling efficiency",
NetResDeep(n_chans1=32, n_blocks=10), per-rank batch 32 (reference main.py:61), SGD lr 1e-2, one process per GPU,
gradient all-reduce = one-shot xGMI peer reads fused with SGD (RCCL fallback).  Synthetic CIFAR-shaped uint8 data (no datasets offline), random-init weights.

Each step is the FULL training step (stem+10 blocks forward, loss, backward, gradient all-reduce, SGD update,
BN running stats) replayed as hipGraphs (16 steps per launch) by the native engine.  W warm-up steps, then K timed steps bracketed by
barrier + device sync on both sides; the slowest rank's time is reported.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype bf16|fp32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

BASELINE_METRIC = "images/sec (whole node) CIFAR-10 ResNet at 1/2/4/8 MI355X; scaling efficiency"
# Practical bar measured this round: the reference training step as-is (PyTorch-ROCm eager + stock DDP,
# host data pipeline) on one MI355X -> profiles/reference_eager_mi355x.log.  BASELINE.md publishes no number.
REF_EAGER_IPS_PER_GPU = 10958.3


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32, help="per-rank batch (reference main.py:61)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--rows", type=int, default=4)
    ap.add_argument("--engine", default="auto", choices=["auto", "persistent", "multikernel"])
    ap.add_argument("--allreduce", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="gradient all-reduce for N>1: one-shot xGMI peer reads (default inside a node) or RCCL")
    a = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        if world == 1 and a.gpus > 1:
            print(f"bench.py: --gpus {a.gpus} needs torch.distributed.run with {a.gpus} processes", file=sys.stderr)
            return 2
    # Rehearsal hook (tests / 1-GPU boxes): DCA_BENCH_SHARE_GPU=1 puts every rank on GPU 0 with a gloo process
    # group (RCCL refuses two ranks per device); the gradient all-reduce is still the engine's xGMI path.
    share = os.environ.get("DCA_BENCH_SHARE_GPU") == "1"
    dev_index = 0 if share else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if share:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from model.resnet import NetResDeep
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer

    data, labels = synthetic_cifar(50000, seed=0)
    torch.manual_seed(1234 + rank)  # ranks init differently; the DDP wrap broadcasts rank 0's weights (CC3)
    model = NetResDeep().to(dev)
    persistent = None if a.engine == "auto" else a.engine == "persistent"
    trainer = FusedDDPTrainer(model, data.to(dev), labels.to(dev), batch_max=a.batch, lr=1e-2, dtype=a.dtype,
                              rows=a.rows, max_indices=(a.warmup + a.steps) * a.batch, persistent=persistent,
                              comm=a.allreduce)
    sampler = torch.utils.data.distributed.DistributedSampler(range(50000), num_replicas=world, rank=rank)
    order = np.resize(np.fromiter(iter(sampler), dtype=np.int32), (a.warmup + a.steps) * a.batch)
    trainer.engine.set_indices(order)
    trainer.engine.set_cursor(0)
    trainer.engine.read_loss(reset=True)

    trainer.engine.run(a.batch, a.warmup)
    trainer.engine.sync()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    trainer.engine.run(a.batch, a.steps)
    trainer.engine.sync()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    dist.barrier()
    t = torch.tensor([dt], device="cpu" if share else dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    loss_sum, nsteps = trainer.engine.read_loss()
    ok = np.isfinite(loss_sum)
    value = world * a.batch * a.steps / dt
    if rank == 0:
        print(json.dumps({
            "metric": BASELINE_METRIC,
            "value": round(value, 1),
            "unit": "images/sec",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(1e3 * dt / a.steps, 5),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": round(value / (REF_EAGER_IPS_PER_GPU * world), 3),
            "dtype": a.dtype,
            "engine": "persistent" if trainer.engine.cfg.persistent else "multikernel",
            "allreduce": trainer.comm,
            "data": "synthetic (CIFAR-10-shaped uint8 3x32x32, 50000 samples, random labels; random-init weights)",
            "config": {"model": "NetResDeep(n_chans1=32, n_blocks=10)", "global_batch": a.batch * world,
                       "per_rank_batch": a.batch, "seq_len": None, "image": "3x32x32",
                       "parallelism": f"dp{world}", "optimizer": "SGD(lr=1e-2)",
                       "baseline": "reference main.py step as-is, PyTorch-ROCm eager on 1x MI355X "
                                   f"({REF_EAGER_IPS_PER_GPU} img/s/GPU, profiles/reference_eager_mi355x.log)"},
            "loss_finite": bool(ok),
            "mean_loss": loss_sum / max(nsteps, 1),
        }), flush=True)
    trainer.close()
    dist.destroy_process_group()
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
