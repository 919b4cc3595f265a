"""ResNet-50 data-parallel training throughput (BASELINE.json extension config: synthetic 3x224x224, DDP).

Generic path of the framework: FlatBucketDDP (flat parameter/gradient buffers, bucketed asynchronous RCCL
all-reduce launched from gradient hooks so it overlaps the backward) + FlatSGD (momentum 0.9, one fused update),
bf16 autocast.  Prints one JSON line (whole-job images/sec, slowest rank).

    python bench/resnet50.py [--batch 256] [--steps 30] [--warmup 5]
    python bench/resnet50.py --gpus 8                      # spawns 8 ranks itself (reference main.py:80-85)
    python bench/resnet50.py --sweep 1,2,4,8               # one fresh rank group per N + scaling efficiency
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 bench/resnet50.py --gpus 8
    python bench/resnet50.py --path torch                  # stock PyTorch (MIOpen convs, channels_last, autocast)
The parent of a self-launch never touches the GPU (ranks are spawned before any HIP call).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--batch", type=int, default=256, help="per-rank batch (288 GB HBM per GPU: large per-GPU batches)")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--image", type=int, default=224)
    ap.add_argument("--bucket-mb", type=float, default=8.0)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--path", default="ops", choices=["torch", "ops"],
                    help="torch: stock conv/BN (MIOpen) under bf16 autocast; ops: the framework's HIP kernels "
                         "(MFMA GEMM convs, fused BN+ReLU+residual, fused CE, HIP SGD)")
    ap.add_argument("--fp8", action="store_true", help="ops path: fp8 e4m3 forward GEMMs for 1x1 convs and fc")
    ap.add_argument("--graph", type=int, default=0,
                    help="1: capture the whole training step (forward, backward, SGD) in a HIP graph and replay it "
                         "(one rank: no collectives inside the capture)")
    ap.add_argument("--overlap-sgd", type=int, default=0,
                    help="1: each gradient bucket's SGD update runs right behind its all-reduce during the backward "
                         "(FlatSGD overlap=True; measured 4.6 %% slower on 1 GPU, where there is no all-reduce to hide "
                         "behind); 0: one SGD step after the backward")
    ap.add_argument("--loopback", action="store_true",
                    help="ops path, --gpus 1: every gradient bucket still runs the xGMI all-reduce kernel on the comm "
                         "stream beside the backward, with the rank as its own only peer (the comm kernels' CU "
                         "pressure measured on one device); reports allreduce_us_per_step")
    ap.add_argument("--infer", action="store_true",
                    help="inference (serving) throughput: eval-mode forward under no_grad, BN with the running "
                         "statistics (ops path: k_bn_eval_stats + k_bn_apply), no backward / optimizer")
    ap.add_argument("--channels-last", type=int, default=1,
                    help="torch path: model and input in channels_last (NHWC) memory format")
    ap.add_argument("--sweep", default=None, metavar="N1,N2,..",
                    help="run each N in a fresh spawned rank group; print per-N lines and a scaling summary")
    ap.add_argument("--result-file", default=None, help=argparse.SUPPRESS)
    return ap.parse_args(argv)


def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def run_rank(a) -> None:
    """One rank (rank / world from the launcher env)."""
    import torch
    import torch.distributed as dist
    import torch.nn.functional as F

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29531")
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
    from distributeddataparallel_cifar10_amd.models.resnet50 import resnet50
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD
    torch.manual_seed(rank)
    model = resnet50().to(dev)
    cl = a.path == "torch" and bool(a.channels_last)
    if cl:
        model = model.to(memory_format=torch.channels_last)
    if a.path == "ops":
        from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
        model = OpsModel(model, fp8=a.fp8)
    if a.path == "torch":  # stock PyTorch end to end: torch DDP + torch.optim.SGD
        ddp = torch.nn.parallel.DistributedDataParallel(model, device_ids=[local])
        opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    else:
        ddp = FlatBucketDDP(model, bucket_cap_mb=a.bucket_mb, first_bucket_mb=1.0, loopback=a.loopback)
        opt = FlatSGD(ddp, lr=0.1, momentum=0.9, overlap=bool(a.overlap_sgd))
    g = torch.Generator(device=dev).manual_seed(1234 + rank)
    x = torch.randn(a.batch, 3, a.image, a.image, device=dev, generator=g)
    if cl:
        x = x.contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 1000, (a.batch,), device=dev, generator=g)
    amp = torch.autocast("cuda", dtype=torch.bfloat16, enabled=a.dtype == "bf16" and a.path == "torch")
    ce = cross_entropy if a.path == "ops" else F.cross_entropy
    one = torch.ones((), device=dev)  # the loss's seed gradient, allocated once (autograd would fill one per step)

    def step():
        if a.infer:
            with torch.no_grad(), amp:
                return model(x).float().logsumexp(1).mean()  # logits consumed on the device, no host sync
        with amp:
            loss = ce(ddp(x), y)
        opt.zero_grad()
        loss.backward(one)
        opt.step()
        return loss

    if a.infer:
        model.eval()

    for _ in range(a.warmup):
        step()
    torch.cuda.synchronize()
    run = step
    if a.graph:
        if world > 1:
            raise SystemExit("--graph: one rank only")
        g_ = torch.cuda.CUDAGraph()
        s_ = torch.cuda.Stream()
        s_.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s_):
            step()  # one more eager step on the capture stream (allocator warm-up)
        torch.cuda.current_stream().wait_stream(s_)
        with torch.cuda.graph(g_):
            static_loss = step()

        def run():
            g_.replay()
            return static_loss
    dist.barrier()
    if hasattr(ddp, "timing") and not a.infer:
        ddp.comm_time(reset=True)
        ddp.timing = True  # comm-stream span per step (first bucket launched -> backward finished)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        loss = run()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    comm_us, comm_n = ddp.comm_time() if getattr(ddp, "timing", False) else (0.0, 0)
    t = torch.tensor([dt], device=dev, dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    if rank == 0:
        v = world * a.batch * a.steps / dt
        metric = ("images/sec (whole node) ResNet-50 synthetic 3x224x224 inference" if a.infer else
                  "images/sec (whole node) ResNet-50 synthetic 3x224x224 DDP")
        print(json.dumps({"metric": metric, "value": round(v, 1), "mode": "inference" if a.infer else "training",
                          "unit": "images/sec", "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
                          "ms_per_step": round(1e3 * dt / a.steps, 3), "higher_is_better": True, "scaling": "weak",
                          "dtype": a.dtype, "data": "synthetic", "loss": float(loss.detach()),
                          "config": {"model": "ResNet-50", "per_rank_batch": a.batch, "image": a.image,
                                     "parallelism": f"dp{world}",
                                     "optimizer": None if a.infer else "SGD(0.1, momentum 0.9)" +
                                     (", per-bucket updates overlapped with the backward" if a.overlap_sgd else ""),
                                     "path": (("eval-mode forward, ops HIP kernels" if a.infer else "FlatBucketDDP + ops HIP kernels") + (" (fp8 fwd GEMMs)" if a.fp8 else " (bf16)")
                                              + (", step replayed as a HIP graph" if a.graph else ""))
                                     if a.path == "ops" else "stock PyTorch: torch DDP + MIOpen convs + torch.optim.SGD, bf16 autocast" +
                                     (", channels_last" if cl else ", NCHW")},
                          "comm": getattr(ddp, "comm", None),
                          # span of the gradient collectives on the comm stream per step (first bucket launched
                          # to backward end: overlapped with the backward, not the exposed cost -- that is the
                          # step-time difference against the run without --loopback)
                          "allreduce_us_per_step": round(comm_us / comm_n, 1) if comm_n else None,
                          "allreduce_metric": "comm-stream span per step (overlapped)" if comm_n else None,
                          "xgmi_calibration": getattr(getattr(ddp, "xgmi", None), "calibration", None)}),
              flush=True)
        if a.result_file:
            with open(a.result_file, "w") as f:
                json.dump({"value": v, "ms_per_step": round(1e3 * dt / a.steps, 3)}, f)
    dist.destroy_process_group()


def _spawned(local_rank: int, world: int, port: int, argv: list) -> None:
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    run_rank(_args(argv))


def main() -> int:
    argv = sys.argv[1:]
    a = _args(argv)
    if a.sweep:
        import torch.multiprocessing as mp
        i = argv.index("--sweep")
        rest = argv[:i] + argv[i + 2:]
        res = {}
        for n in [int(x) for x in a.sweep.split(",")]:
            with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
                path = f.name
            mp.spawn(_spawned, args=(n, _free_port(), rest + ["--gpus", str(n), "--result-file", path]), nprocs=n,
                     join=True)
            with open(path) as f:
                res[n] = json.load(f)
            os.unlink(path)
        n0 = min(res)
        base = res[n0]["value"] / n0
        print(json.dumps({"metric": "images/sec (whole node) ResNet-50 synthetic 3x224x224 DDP",
                          "sweep": {str(n): round(r["value"], 1) for n, r in res.items()},
                          "scaling_efficiency": {str(n): round(r["value"] / (n * base), 4) for n, r in res.items()},
                          "ms_per_step": {str(n): r["ms_per_step"] for n, r in res.items()}}), flush=True)
        return 0
    if "WORLD_SIZE" in os.environ:  # started by torch.distributed.run
        if int(os.environ["WORLD_SIZE"]) != a.gpus:
            print(f"resnet50.py: --gpus {a.gpus} but the launcher started {os.environ['WORLD_SIZE']} ranks",
                  file=sys.stderr)
            return 2
        run_rank(a)
        return 0
    if a.loopback and (a.gpus != 1 or a.path != "ops" or a.graph):
        print("resnet50.py: --loopback needs --gpus 1 --path ops (no --graph)", file=sys.stderr)
        return 2
    if a.gpus == 1:
        os.environ.setdefault("WORLD_SIZE", "1")
        run_rank(a)
        return 0
    import torch.multiprocessing as mp
    mp.spawn(_spawned, args=(a.gpus, _free_port(), argv), nprocs=a.gpus, join=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
