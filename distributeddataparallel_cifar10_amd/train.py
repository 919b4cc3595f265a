"""Training application shared by ``main.py`` (DDP) and ``main_no_ddp.py`` (single device).

Reference: ``main.py:26-65`` (``train_loop``, ``main``) and ``main_no_ddp.py:22-63`` (``prepare``,
``training_loop``).  Defaults reproduce the reference exactly -- SGD(lr=1e-2), CrossEntropyLoss, epochs 1..99,
per-rank batch 32 with DistributedSampler order (no set_epoch), log + checkpoint at epoch 1 and every 10th epoch,
the same stdout lines -- while the step itself runs on the MI355X-native path:

* ``engine="fused"`` (default on a GPU, NetResDeep): the whole step (forward, loss, backward, gradient
  all-reduce -- one-shot xGMI peer reads or RCCL --, SGD, BN running stats) is ONE hipGraph replay of the native engine; the dataset is
  device-resident; the loss is accumulated on the device and read once per epoch (reference ``loss.item()``
  every step, SURVEY.md Q9: same printed value, no per-step host sync).
* ``engine="ops"``: the framework's general HIP layer kernels (``ops/``: MFMA GEMM convolutions, fused
  BN + ReLU + residual, fused cross-entropy, HIP SGD; fp8 forward GEMMs with ``fp8``) + ``FlatBucketDDP``.
* ``engine="torch"``: stock PyTorch ops + ``FlatBucketDDP`` (generic path; CPU / gloo; any model).

Options beyond the reference (all off by default): max_steps (per epoch), synthetic data, resume, metrics JSON,
fault injection (``fail_at_step``), process-group timeout, set_epoch reshuffling, bf16/fp32 engine precision.
"""
from __future__ import annotations

import argparse
import os
import time
from dataclasses import dataclass, field
from typing import Optional

import torch
import torch.nn as nn

from .data.cifar import load_cifar10
from .data.loader import DeviceLoader
from .data.synthetic import synthetic_cifar
from .utils.checkpoint import CHECKPOINT_NAME, load_checkpoint, save_checkpoint, unwrap
from .utils.metrics import MetricsLog, epoch_line, should_log, time_line


@dataclass
class TrainConfig:
    epochs: int = 99                 # range(1, 100) (reference main.py:30)
    lr: float = 1e-2                 # reference main.py:27
    batch_size: int = 32             # reference main.py:61 (main_no_ddp.py:31 hard-codes 64)
    data_path: str = "data/CIFAR-10/"
    synthetic: int = 0               # >0: use N synthetic CIFAR-shaped samples instead of the dataset
    synthetic_learnable: bool = False  # synthetic "hard" learnable set (data/synthetic.py: blended class colour,
                                       # random-phase class stripes under noise, 10 % label noise)
    engine: str = "auto"             # auto | fused | torch
    dtype: str = "fp32"              # compute precision: fp32 = the reference's numerics (default), bf16 = MFMA bf16
    max_steps: Optional[int] = None  # per-epoch step cap (smoke tests / benchmarking)
    checkpoint: bool = True
    checkpoint_path: Optional[str] = None
    resume: Optional[str] = None
    metrics_json: Optional[str] = None
    seed: int = 0
    set_epoch: bool = False
    fail_at_step: Optional[int] = None
    backend: str = "nccl"
    port: Optional[int] = None
    timeout_s: Optional[float] = None
    model: str = "netresdeep"        # netresdeep | resnet50 (generic path)
    bucket_mb: float = 4.0           # FlatBucketDDP bucket cap (generic path)
    profile: Optional[str] = None    # directory for torch.profiler traces / kernel summary
    check_sync: int = 0              # >0: assert cross-rank parameter equality every N epochs (and at start)
    allreduce: str = "auto"          # fused engine gradient all-reduce: auto | xgmi (one-shot P2P) | rccl
    fp8: bool = False                # ops engine: fp8 e4m3 forward GEMMs for 1x1 convs / fc (ResNet family)
    extra: dict = field(default_factory=dict)


def add_cli_args(ap: argparse.ArgumentParser, batch_default: int = 32) -> argparse.ArgumentParser:
    ap.add_argument("--epochs", type=int, default=99)
    ap.add_argument("--max-steps", type=int, default=None, help="cap on steps per epoch")
    ap.add_argument("--batch-size", type=int, default=batch_default)
    ap.add_argument("--lr", type=float, default=1e-2)
    ap.add_argument("--data-root", default=None)
    ap.add_argument("--synthetic", type=int, nargs="?", const=50000, default=0,
                    help="train on N synthetic CIFAR-shaped samples (default 50000)")
    ap.add_argument("--synthetic-learnable", action="store_true",
                    help="synthetic data whose label is a function of the image (blended class colour + random-phase "
                         "class stripes under noise, 10%% label noise), so the loss has a learning curve; implies "
                         "--synthetic 50000 unless given")
    ap.add_argument("--engine", default="auto", choices=["auto", "fused", "ops", "torch"],
                    help="fused: NetResDeep native engine; ops: the framework's HIP layer kernels (any supported "
                         "model) + FlatBucketDDP; torch: stock PyTorch ops + FlatBucketDDP")
    ap.add_argument("--fp8", action="store_true", help="ops engine: fp8 e4m3 forward GEMMs (1x1 convs, fc)")
    ap.add_argument("--dtype", default="fp32", choices=["bf16", "fp32"],
                    help="fp32 (default): fp32-accurate, the reference's dtype (the sliced engine computes every "
                         "product as 3 bf16 MFMA products, ~2^-17 relative error; the multi-kernel engine exact fp32 "
                         "MFMA); bf16: bf16 MFMA operands, fp32 accumulation")
    ap.add_argument("--no-checkpoint", action="store_true")
    ap.add_argument("--checkpoint-path", default=None)
    ap.add_argument("--resume", default=None)
    ap.add_argument("--metrics-json", default=None)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--set-epoch", action="store_true", help="reshuffle every epoch (reference never does)")
    ap.add_argument("--fail-at-step", type=int, default=None, help="fault injection: raise on this global step")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"])
    ap.add_argument("--world-size", type=int, default=None, help="number of ranks (default: GPU count)")
    ap.add_argument("--port", type=int, default=None)
    ap.add_argument("--timeout", type=float, default=None, help="process-group timeout in seconds")
    ap.add_argument("--model", default="netresdeep", choices=["netresdeep", "resnet50"])
    ap.add_argument("--bucket-mb", type=float, default=4.0, help="gradient bucket cap (generic DDP path)")
    ap.add_argument("--profile", default=None, metavar="DIR", help="write torch.profiler traces to DIR")
    ap.add_argument("--check-sync", type=int, default=0, metavar="N",
                    help="assert parameters are identical on all ranks at start and every N epochs")
    ap.add_argument("--allreduce", default="auto", choices=["auto", "xgmi", "rccl"],
                    help="fused engine gradient all-reduce: one-shot xGMI peer reads (auto inside a node) or RCCL")
    return ap


def config_from_args(a: argparse.Namespace, data_path_default: str) -> TrainConfig:
    learnable = bool(getattr(a, "synthetic_learnable", False))
    return TrainConfig(epochs=a.epochs, lr=a.lr, batch_size=a.batch_size, data_path=a.data_root or data_path_default,
                       synthetic=a.synthetic or (50000 if learnable else 0), synthetic_learnable=learnable,
                       engine=a.engine, dtype=a.dtype, max_steps=a.max_steps,
                       checkpoint=not a.no_checkpoint, checkpoint_path=a.checkpoint_path, resume=a.resume,
                       metrics_json=a.metrics_json, seed=a.seed, set_epoch=a.set_epoch, fail_at_step=a.fail_at_step,
                       backend=a.backend, port=a.port, timeout_s=a.timeout, model=a.model, bucket_mb=a.bucket_mb,
                       profile=a.profile, check_sync=a.check_sync, allreduce=a.allreduce, fp8=a.fp8)


def load_dataset(cfg: TrainConfig):
    if cfg.synthetic:
        return synthetic_cifar(cfg.synthetic, seed=cfg.seed, learnable="hard" if cfg.synthetic_learnable else False)
    return load_cifar10(cfg.data_path, train=True)


FUSED_BATCH_MAX = 64  # csrc/common.h BMAX_LIMIT: per-rank batch the fused NetResDeep engine supports


def resolve_engine(cfg: TrainConfig, device: torch.device, model: nn.Module) -> str:
    """auto: NetResDeep on the fused engine (per-rank batch <= 64), other models (ResNet family) and larger
    NetResDeep batches on the ops-layer HIP kernels, on a GPU; stock torch ops on the CPU."""
    if cfg.engine == "fused" and cfg.batch_size > FUSED_BATCH_MAX:
        raise ValueError(f"--engine fused supports --batch-size <= {FUSED_BATCH_MAX} per rank "
                         f"(got {cfg.batch_size}); use --engine ops or auto")
    if cfg.engine != "auto":
        return cfg.engine
    if device.type != "cuda":
        return "torch"
    return "fused" if _is_netresdeep(model) and cfg.batch_size <= FUSED_BATCH_MAX else "ops"


def _is_netresdeep(model: nn.Module) -> bool:
    return getattr(model, "n_chans1", None) == 32 and getattr(model, "n_blocks", None) == 10


class _Fault(RuntimeError):
    pass


def train_loop(model, train_loader: DeviceLoader, rank: int, cfg: Optional[TrainConfig] = None,
               optimizer=None) -> dict:
    """Reference ``main.py:26-49`` / ``main_no_ddp.py:36-59``.  `model` is a ``FusedDDPTrainer`` (engine path),
    a ``FlatBucketDDP`` or a plain module (torch path).  Returns a summary dict."""
    from .parallel.ddp import FusedDDPTrainer
    cfg = cfg or TrainConfig()
    mlog = MetricsLog(cfg.metrics_json, rank)
    ckpt = cfg.checkpoint_path or os.path.join(cfg.data_path, CHECKPOINT_NAME)
    fused = isinstance(model, FusedDDPTrainer)
    n_batches = len(train_loader)
    steps_per_epoch = min(n_batches, cfg.max_steps) if cfg.max_steps else n_batches
    start_epoch = int(cfg.extra.get("start_epoch", 1))
    global_step = int(cfg.extra.get("start_step", 0))
    history = []
    from .ops.models import OpsModel
    on_ops = isinstance(getattr(model, "module", None), OpsModel)
    if not fused:
        loss_fn = nn.CrossEntropyLoss()
        if on_ops:
            from .ops.functional import cross_entropy as loss_fn
        if optimizer is None:
            from .parallel.flat_ddp import FlatBucketDDP, FlatSGD
            optimizer = FlatSGD(model, cfg.lr) if isinstance(model, FlatBucketDDP) else \
                torch.optim.SGD(model.parameters(), lr=cfg.lr)
    from contextlib import ExitStack
    from .utils.trace import trace_range as record_function  # torch.profiler + roctx ranges
    from .parallel.dist import assert_params_in_sync
    autocast = (not fused and not on_ops and cfg.dtype == "bf16" and train_loader.device.type == "cuda"
                and not _is_netresdeep(unwrap(model)))  # generic models train in bf16; NetResDeep torch path = fp32
    if cfg.check_sync:
        assert_params_in_sync(unwrap(model))
    if cfg.metrics_json and hasattr(model, "timing"):
        model.timing = True  # FlatBucketDDP: record the comm-stream span per step
    if cfg.metrics_json and fused:
        model.engine.comm_time(reset=True)
    stack = ExitStack()
    prof = stack.enter_context(_profiler(cfg.profile, train_loader.device)) if cfg.profile else None
    start_time = time.time()
    for epoch in range(start_epoch, cfg.epochs + 1):
        train_loader.set_epoch(epoch)
        t0 = time.perf_counter()
        if fused:
            bs = train_loader.batch_size
            idx = train_loader.indices()[:steps_per_epoch * bs]
            if cfg.fail_at_step is not None and global_step < cfg.fail_at_step <= global_step + steps_per_epoch:
                done = cfg.fail_at_step - global_step - 1  # steps before the failing one still run, as on the
                if done:                                   # generic path (the failure is raised AT that step)
                    model.engine.run_epoch(idx[:done * bs], bs)
                raise _Fault(f"injected failure at step {cfg.fail_at_step} (rank {rank})")
            with record_function(f"epoch{epoch}:engine"):
                loss_sum, nsteps = model.engine.run_epoch(idx, bs)
        else:
            loss_sum, nsteps = 0.0, 0
            for imgs, labels in train_loader:
                if nsteps >= steps_per_epoch:
                    break
                if cfg.fail_at_step is not None and global_step + nsteps + 1 == cfg.fail_at_step:
                    raise _Fault(f"injected failure at step {cfg.fail_at_step} (rank {rank})")
                with record_function("forward"), torch.autocast("cuda", torch.bfloat16, enabled=autocast):
                    outputs = model(imgs)
                    loss = loss_fn(outputs.float(), labels)
                optimizer.zero_grad()
                with record_function("backward+allreduce"):
                    loss.backward(_seed_grad(loss))
                with record_function("optimizer"):
                    optimizer.step()
                loss_sum += loss.item()
                nsteps += 1
        global_step += nsteps
        dt = time.perf_counter() - t0
        if hasattr(model, "check_comm"):  # a peer timeout of the xGMI all-reduce must not go unnoticed
            model.check_comm()            # (rank-divergent gradients): raise before anything is saved
        mean = loss_sum / n_batches  # reference divides by len(train_loader) (main.py:44)
        history.append(mean)
        comm_us, comm_n = _comm_time(model) if cfg.metrics_json else (0.0, 0)
        eng = getattr(model, "engine", None)
        mlog.write(epoch=epoch, loss=mean, steps=nsteps, seconds=dt, step_ms=1e3 * dt / max(nsteps, 1),
                   images_per_sec=nsteps * train_loader.batch_size / max(dt, 1e-9),
                   # exposed wait of the reduction kernel's gradient-segment exchanges, summed per step (xGMI)
                   allreduce_us_per_step=(comm_us / comm_n) if comm_n else None,
                   engine=getattr(eng, "kind_name", cfg.engine if not fused else None),
                   dtype=cfg.dtype, fp32_mode=("3xbf16" if getattr(eng, "kind_name", "") == "sliced" else
                                               "fp32-mfma") if cfg.dtype == "fp32" and fused else None)
        if should_log(epoch):
            print(epoch_line(epoch, mean), flush=True)
            if cfg.checkpoint:
                save_checkpoint(model, ckpt, rank, meta={"epoch": epoch, "step": global_step})
        if cfg.check_sync and epoch % cfg.check_sync == 0:
            assert_params_in_sync(unwrap(model))
    total = time.time() - start_time
    stack.close()
    if prof is not None:
        _export_profile(prof, cfg.profile, rank, train_loader.device)
    print(time_line(total), flush=True)
    # end-of-run record (metrics JSON only): the BN step counter after the last epoch -- the last checkpoint is the
    # epoch-90 one (reference main.py:43-45), so the file holds an earlier count
    nbt = _num_batches_tracked(unwrap(model))
    mlog.write(final=True, steps_total=global_step, seconds_total=total, num_batches_tracked=nbt)
    return {"losses": history, "seconds": total, "steps": global_step, "num_batches_tracked": nbt}


def _num_batches_tracked(module) -> Optional[int]:
    for name, buf in module.named_buffers():
        if name.endswith("num_batches_tracked"):
            return int(buf.item())
    return None


_SEEDS = {}


def _seed_grad(loss: torch.Tensor) -> torch.Tensor:
    """The scalar loss's seed gradient (1.0), allocated once per device and dtype: ``loss.backward()`` would launch
    a fill kernel for it every step."""
    key = (loss.device, loss.dtype)
    if key not in _SEEDS:
        _SEEDS[key] = torch.ones((), device=loss.device, dtype=loss.dtype)
    return _SEEDS[key]


def _comm_time(model) -> tuple:
    """(microseconds, steps) spent in the gradient all-reduce since the last call (per-rank metric)."""
    from .parallel.ddp import FusedDDPTrainer
    if isinstance(model, FusedDDPTrainer):
        return model.engine.comm_time(reset=True)
    if hasattr(model, "comm_time"):
        return model.comm_time(reset=True)
    return 0.0, 0


def _profiler(out_dir: str, device: torch.device):
    """torch.profiler over the training loop (CPU ops + HIP kernels through roctracer on ROCm)."""
    from torch.profiler import ProfilerActivity, profile
    acts = [ProfilerActivity.CPU] + ([ProfilerActivity.CUDA] if device.type == "cuda" else [])
    os.makedirs(out_dir, exist_ok=True)
    return profile(activities=acts, record_shapes=False)


def _export_profile(prof, out_dir: str, rank: int, device: torch.device) -> None:
    prof.export_chrome_trace(os.path.join(out_dir, f"trace_rank{rank}.json"))
    key = "self_cuda_time_total" if device.type == "cuda" else "self_cpu_time_total"
    with open(os.path.join(out_dir, f"summary_rank{rank}.txt"), "w") as f:
        f.write(prof.key_averages().table(sort_by=key, row_limit=40))


def build_model_for_rank(cfg: TrainConfig, rank: int, world_size: int, device: torch.device, data, labels,
                         loader: DeviceLoader):
    """The model wrapped for data parallelism on `device`: NetResDeep on the fused engine, or any model on
    FlatBucketDDP (``--model resnet50`` trains a 10-class ResNet-50 on the CIFAR tensors, channels-last, bf16)."""
    from .models.netresdeep import NetResDeep
    from .parallel.ddp import FusedDDPTrainer
    from .parallel.flat_ddp import FlatBucketDDP
    if cfg.model == "resnet50":
        from .models.resnet50 import resnet50
        torch.manual_seed(cfg.seed)
        model = resnet50(num_classes=10).to(device)
        if device.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        if cfg.engine == "fused":
            raise ValueError("the fused engine implements NetResDeep only; use --engine ops/torch/auto for resnet50")
    else:
        model = NetResDeep().to(device)
    meta = None
    if cfg.resume:
        meta = load_checkpoint(model, cfg.resume, strict=True, map_location=device)
        if meta:
            cfg.extra["start_epoch"] = int(meta.get("epoch", 0)) + 1
            cfg.extra["start_step"] = int(meta.get("step", 0))
    kind = resolve_engine(cfg, device, model)
    if kind == "ops":
        from .ops.models import OpsModel
        if device.type != "cuda":
            raise ValueError("--engine ops runs the HIP kernels: it needs a GPU")
        return FlatBucketDDP(OpsModel(model, fp8=cfg.fp8), bucket_cap_mb=cfg.bucket_mb)
    if kind == "fused":
        n_idx = len(loader) * loader.batch_size
        return FusedDDPTrainer(model, loader.data, loader.labels, batch_max=loader.batch_size, lr=cfg.lr,
                               dtype=cfg.dtype, max_indices=max(n_idx, loader.batch_size), comm=cfg.allreduce)
    return FlatBucketDDP(model, bucket_cap_mb=cfg.bucket_mb)

