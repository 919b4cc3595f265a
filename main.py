"""DDP training of NetResDeep on CIFAR-10, one process per MI355X (reference ``main.py``).

Same entry point, function names and default behaviour as the reference:
    python main.py            # world_size = number of visible GPUs, mp.spawn one rank per GPU
prints ``Using N GPUs`` (N>1), ``Epoch {e}, Training loss {x}`` at epoch 1 and every 10th epoch, and
``training time: {s:.3f} seconds``; rank 0 writes ``data/CIFAR-10/birds_vs_airplanes.pt`` at the same epochs.

The step runs on the native MI355X engine (HIP/CDNA4 kernels, hipGraph replay; the gradient all-reduce is the
in-kernel xGMI exchange by default, RCCL with ``--allreduce rccl``);
``--engine torch`` selects the generic stock-op path.  Every flag is optional (see --help); without flags the
behaviour is the reference's.  With no GPU, nothing runs unless ``--backend gloo --world-size N`` asks for CPU
ranks (reference: 0 GPUs -> mp.spawn(nprocs=0) silently does nothing).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch
import torch.multiprocessing as mp

from distributeddataparallel_cifar10_amd.data.loader import DeviceLoader
from distributeddataparallel_cifar10_amd.parallel import dist as pdist
from distributeddataparallel_cifar10_amd.train import (TrainConfig, add_cli_args, build_model_for_rank,
                                                       config_from_args, load_dataset)
from distributeddataparallel_cifar10_amd.train import train_loop as _train_loop
from distributeddataparallel_cifar10_amd.utils.gpu import free_gpu_cache  # noqa: F401  (reference main.py:67)

data_path = 'data/CIFAR-10/'  # reference main.py:19


def setup(rank, world_size, backend="nccl", port=None, timeout_s=None):
    """Reference main.py:21-24 (RCCL process group; the GPU is bound explicitly)."""
    pdist.setup(rank, world_size, backend=backend, port=port, timeout_s=timeout_s)


def train_loop(model, train_loader, rank, cfg=None):
    """Reference main.py:26-49."""
    return _train_loop(model, train_loader, rank, cfg or TrainConfig(data_path=data_path))


def main(rank, world_size, cfg=None):
    """Reference main.py:51-65 (per-process entry)."""
    cfg = cfg or TrainConfig(data_path=data_path)
    setup(rank, world_size, cfg.backend, cfg.port, cfg.timeout_s)
    try:
        device = torch.device("cuda", rank) if cfg.backend == "nccl" else torch.device("cpu")
        data, labels = load_dataset(cfg)
        loader = DeviceLoader(data, labels, batch_size=cfg.batch_size, world_size=world_size, rank=rank,
                              device=device, sampler="distributed", seed=0, set_epoch=cfg.set_epoch)
        model = build_model_for_rank(cfg, rank, world_size, device, data, labels, loader)
        train_loop(model, train_loader=loader, rank=rank, cfg=cfg)
        if hasattr(model, "close"):
            model.close()
    finally:
        pdist.teardown()


def _parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    add_cli_args(ap, batch_default=32)
    return ap.parse_args(argv)


if __name__ == '__main__':
    args = _parse()
    cfg = config_from_args(args, data_path)
    if args.backend == "gloo":
        world_size = args.world_size or 1
    else:
        if torch.cuda.device_count() > 1:
            print("Using", torch.cuda.device_count(), "GPUs")
        world_size = args.world_size or torch.cuda.device_count()
    os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    mp.spawn(main, args=(world_size, cfg), nprocs=world_size)
    sys.exit(0)
