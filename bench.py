"""Headline benchmark: whole-node images/sec of NetResDeep CIFAR-10 DDP training on MI355X.

Metric/config from BASELINE.json: "images/sec (whole node) CIFAR-10 ResNet at 1/2/4/8 MI355X; scaling efficiency",
NetResDeep(n_chans1=32, n_blocks=10), per-rank batch 32 (reference main.py:61), SGD lr 1e-2, one process per GPU,
gradient all-reduce = one-shot xGMI peer reads fused with SGD (RCCL fallback).  Synthetic CIFAR-shaped uint8 data
(no datasets offline), random-init weights.

Each step is the FULL training step (stem + 10 blocks forward, loss, backward, gradient all-reduce, SGD update,
BN running stats) replayed as hipGraphs (16 steps per launch) by the native engine.  The graphs are captured during
warm-up (never inside the timed region).  W warm-up steps, then K timed steps bracketed by barrier + device sync on
both sides; the slowest rank's time is reported.

Launch modes (reference main.py:80-85 launches its ranks itself with mp.spawn; so does this):
    python bench.py [--gpus N] [--steps K] [--warmup W] [--dtype bf16|fp32]     # N>1: spawns N ranks itself
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 --master-port P bench.py --gpus N
    python bench.py --sweep 1,2,4,8                                               # one fresh rank group per N,
                                                                                  # + scaling-efficiency summary
The parent of a self-launch never touches the GPU (ranks are spawned before any HIP call).
DCA_BENCH_SHARE_GPU=1 (rehearsal on a 1-GPU box): every rank on GPU 0, gloo process group, xGMI all-reduce.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

# Cross-process GPU memory sharing (the xGMI all-reduce maps each peer's gradient region with hipIpcOpenMemHandle;
# RCCL's intra-node transport shares buffers the same way) must use the dmabuf IPC path: the hosts' kernel driver
# supports only dmabuf, and with the legacy IPC mode hipIpcGetMemHandle fails with "invalid argument"
# (profiles/ipc_mode_legacy_r7.log).  Set before any HIP call of this process and inherited by every spawned or
# torchrun-started rank; an explicit setting in the caller's environment wins.  Same rule: main.py, ppe_main_ddp.py.
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")

BASELINE_METRIC = "images/sec (whole node) CIFAR-10 ResNet at 1/2/4/8 MI355X; scaling efficiency"
# Practical bar (BASELINE.md publishes no number): the reference training step as-is -- PyTorch-ROCm eager + stock
# DDP + its host data pipeline -- on one MI355X, measured per precision (bench/reference_eager.py):
#   fp32 (the reference's own precision): profiles/reference_eager_mi355x.log
#   bf16 (the same step under torch.autocast bf16): profiles/reference_eager_bf16_mi355x.log
REF_EAGER_IPS_PER_GPU = {"fp32": 10958.3, "bf16": 10207.4}


def _args(argv=None):
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
    ap.add_argument("--loopback", action="store_true",
                    help="--gpus 1 --allreduce xgmi: run the xGMI gradient exchange with the rank as its own only peer "
                         "(protocol cost on one device; not the headline configuration)")
    ap.add_argument("--sweep", default=None, metavar="N1,N2,..",
                    help="run each N in a fresh spawned rank group; print per-N lines and a scaling summary")
    ap.add_argument("--no-fp32", action="store_true",
                    help="bf16 runs: skip the second, fp32 (reference precision) timing in the same invocation")
    ap.add_argument("--result-file", default=None, help=argparse.SUPPRESS)  # rank 0 -> parent (sweep)
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_rank(a) -> dict | None:
    """One rank of the benchmark (rank / world from the launcher env).  Returns rank 0's result dict."""
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    share = os.environ.get("DCA_BENCH_SHARE_GPU") == "1"
    dev_index = 0 if share else local_rank
    torch.cuda.set_device(dev_index)
    dev = torch.device("cuda", dev_index)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29511")
    if share:  # RCCL refuses two ranks per device; the gradient all-reduce is still the engine's xGMI path
        dist.init_process_group("gloo", rank=rank, world_size=world)
    else:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    from model.resnet import NetResDeep
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer

    data, labels = synthetic_cifar(50000, seed=0)
    data, labels = data.to(dev), labels.to(dev)
    sampler = torch.utils.data.distributed.DistributedSampler(range(50000), num_replicas=world, rank=rank)
    order = np.resize(np.fromiter(iter(sampler), dtype=np.int32), (a.warmup + a.steps) * a.batch)

    def timed(dtype: str):
        """W warm-up + K timed steps of a fresh model / engine in `dtype`; the slowest rank's seconds."""
        torch.manual_seed(1234 + rank)  # ranks init differently; the DDP wrap broadcasts rank 0's weights (CC3)
        model = NetResDeep().to(dev)
        persistent = None if a.engine == "auto" else a.engine == "persistent"
        trainer = FusedDDPTrainer(model, data, labels, batch_max=a.batch, lr=1e-2, dtype=dtype, rows=a.rows,
                                  max_indices=(a.warmup + a.steps) * a.batch, persistent=persistent,
                                  comm=a.allreduce, loopback=a.loopback)
        eng = trainer.engine
        eng.set_indices(order)
        eng.set_cursor(0)
        eng.precapture(a.batch)  # graph capture + instantiate happen here, outside the timed region
        eng.read_loss(reset=True)
        eng.run(a.batch, a.warmup)
        eng.sync()
        eng.comm_time(reset=True)
        dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        eng.run(a.batch, a.steps)
        eng.sync()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        dist.barrier()
        comm_us, comm_calls = eng.comm_time()
        on = "cpu" if share else dev
        mine = torch.tensor([dt, comm_us / max(comm_calls, 1)], device=on, dtype=torch.float64)
        every = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(every, mine)
        per_rank = [(float(t[0].item()), float(t[1].item())) for t in every]
        loss_sum, nsteps = eng.read_loss()
        out = {"dt": max(p[0] for p in per_rank), "per_rank": per_rank, "loss": loss_sum / max(nsteps, 1),
               "ok": bool(np.isfinite(loss_sum)), "engine": eng.kind_name, "comm": trainer.comm}
        trainer.close()
        return out

    main_run = timed(a.dtype)
    dt, per_rank, ok = main_run["dt"], main_run["per_rank"], main_run["ok"]
    value = world * a.batch * a.steps / dt
    ref = REF_EAGER_IPS_PER_GPU.get(a.dtype)
    res = {
        "metric": BASELINE_METRIC,
        "value": round(value, 1),
        "unit": "images/sec",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(1e3 * dt / a.steps, 5),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (ref * world), 3) if ref else None,
        "dtype": a.dtype,
        "engine": main_run["engine"],
        "allreduce": main_run["comm"],
        "per_rank_ms_per_step": [round(1e3 * p[0] / a.steps, 5) for p in per_rank],
        # exposed gradient-exchange wait per step: the mean wait of one trunk / conv1 segment exchange (they run in
        # parallel on the reduction's critical path; xGMI path only)
        "allreduce_us_per_step": ([round(p[1], 2) for p in per_rank] if main_run["comm"].startswith("xgmi")
                                  else None),
        "data": "synthetic (CIFAR-10-shaped uint8 3x32x32, 50000 samples, random labels; random-init weights)",
        "config": {"model": "NetResDeep(n_chans1=32, n_blocks=10)", "global_batch": a.batch * world,
                   "per_rank_batch": a.batch, "seq_len": None, "image": "3x32x32",
                   "parallelism": f"dp{world}", "optimizer": "SGD(lr=1e-2)",
                   "baseline": (f"reference main.py step as-is, PyTorch-ROCm eager ({a.dtype}) on 1x MI355X, "
                                f"{ref} img/s/GPU (bench/reference_eager.py)") if ref else
                               f"no {a.dtype} reference measurement"},
        "loss_finite": ok,
        "mean_loss": main_run["loss"],
    }
    if a.dtype == "bf16" and not a.no_fp32:
        # the reference's precision, timed in the same invocation (same steps / warm-up / ranks).  The sliced
        # engine's fp32 is "3xbf16": every MFMA operand split into bf16 hi + lo, products hi*hi + hi*lo + lo*hi,
        # fp32 accumulation / BatchNorm / loss / SGD (measured against the fp32 oracle: tests/test_engine_gpu.py)
        f = timed("fp32")
        fv = world * a.batch * a.steps / f["dt"]
        res.update({"fp32_value": round(fv, 1), "fp32_ms_per_step": round(1e3 * f["dt"] / a.steps, 5),
                    "fp32_mode": "3xbf16" if f["engine"] == "sliced" else "fp32-mfma",
                    "fp32_engine": f["engine"], "fp32_vs_baseline": round(fv / (REF_EAGER_IPS_PER_GPU["fp32"] * world), 3),
                    "fp32_loss_finite": f["ok"]})
        ok = ok and f["ok"]
    if rank == 0:
        print(json.dumps(res), flush=True)
        if a.result_file:
            with open(a.result_file, "w") as f:
                json.dump(res, f)
    dist.destroy_process_group()
    if not ok:
        raise SystemExit(1)
    return res if rank == 0 else None


def _spawned(local_rank: int, world: int, port: int, argv: list) -> None:
    """mp.spawn target: one rank of a self-launched group (reference main.py:84 mp.spawn(main, nprocs=...))."""
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run_rank(_args(argv))


def launch(n: int, argv: list) -> None:
    """Run an n-rank group: in this process for n == 1, else as n spawned processes (no GPU call in the parent)."""
    if n == 1:
        os.environ.setdefault("WORLD_SIZE", "1")
        run_rank(_args(argv))
        return
    import torch.multiprocessing as mp
    _share_queues()
    mp.spawn(_spawned, args=(n, _free_port(), argv), nprocs=n, join=True)


def _share_queues() -> None:
    """Shared-GPU rehearsal: one hardware queue per rank process (inherited at spawn).  Eight processes with the
    default four queues each oversubscribe the device's hardware scheduler, which then time-slices the queues and
    stalls the ranks' spinning exchange kernels (tests/_ranks.py)."""
    if os.environ.get("DCA_BENCH_SHARE_GPU") == "1":
        os.environ["GPU_MAX_HW_QUEUES"] = "1"


def sweep(ns: list, argv: list) -> int:
    """One fresh rank group per N (1-rank groups too run in a child, so every N starts from a clean process)."""
    import torch.multiprocessing as mp
    _share_queues()
    results = {}
    for n in ns:
        with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
            path = f.name
        sub = argv + ["--gpus", str(n), "--result-file", path]
        mp.spawn(_spawned, args=(n, _free_port(), sub), nprocs=n, join=True)
        with open(path) as f:
            results[n] = json.load(f)
        os.unlink(path)
    base = results[min(results)]["value"] / min(results)
    fp32 = {str(n): r["fp32_value"] for n, r in results.items() if "fp32_value" in r}
    print(json.dumps({"metric": BASELINE_METRIC, "sweep": {str(n): r["value"] for n, r in results.items()},
                      **({"fp32_sweep": fp32} if fp32 else {}),
                      "scaling_efficiency": {str(n): round(r["value"] / (n * base), 4) for n, r in results.items()},
                      "ms_per_step": {str(n): r["ms_per_step"] for n, r in results.items()},
                      "dtype": results[min(results)]["dtype"], "unit": "images/sec"}), flush=True)
    return 0


def main() -> int:
    argv = sys.argv[1:]
    a = _args(argv)
    if a.loopback and (a.gpus != 1 or a.allreduce != "xgmi"):
        print("bench.py: --loopback needs --gpus 1 --allreduce xgmi", file=sys.stderr)
        return 2
    if a.sweep:
        rest, skip = [], False
        for x in argv:  # drop both "--sweep N1,N2" and "--sweep=N1,N2"
            if skip:
                skip = False
            elif x == "--sweep":
                skip = True
            elif not x.startswith("--sweep="):
                rest.append(x)
        return sweep([int(x) for x in a.sweep.split(",")], rest)
    if "WORLD_SIZE" in os.environ:  # started by torch.distributed.run (or another launcher)
        world = int(os.environ["WORLD_SIZE"])
        if world != a.gpus:
            print(f"bench.py: --gpus {a.gpus} but the launcher started {world} ranks", file=sys.stderr)
            return 2
        run_rank(a)
        return 0
    launch(a.gpus, argv)
    return 0


if __name__ == "__main__":
    sys.exit(main())
