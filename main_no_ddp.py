"""Single-device training of NetResDeep on CIFAR-10 (reference ``main_no_ddp.py``).

Reference behaviour kept: ``data_path='../data/CIFAR-10/'``, device = GPU if available else CPU with the
``Training on device ...`` line, ``prepare()`` building a batch-64 shuffled loader (its arguments are ignored, as
in the reference) and printing ``len(train_loader)`` (782), ``training_loop(model, train_loader)`` with SGD 1e-2,
CrossEntropyLoss, 99 epochs, the same log lines, no checkpoint.

Deliberate deviation: the reference trains at import time (module-level driver without a ``__main__`` guard);
here the driver runs only when executed as a script, so the functions can be imported.

On a GPU the step runs on the native engine (NetResDeep: device-resident data, one hipGraph replay per step) or
on the ops-layer HIP kernels (other models, ``--engine ops``); on the CPU it runs stock PyTorch ops.  Optional flags: see --help.
"""
from __future__ import annotations

import argparse

import torch

from distributeddataparallel_cifar10_amd.data.loader import DeviceLoader
from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
from distributeddataparallel_cifar10_amd.train import TrainConfig, add_cli_args, config_from_args, load_dataset
from distributeddataparallel_cifar10_amd.train import resolve_engine
from distributeddataparallel_cifar10_amd.train import train_loop as _train_loop

data_path = '../data/CIFAR-10/'  # reference main_no_ddp.py:17
device = (torch.device('cuda') if torch.cuda.is_available()
          else torch.device('cpu'))

_cfg = TrainConfig(data_path=data_path, batch_size=64, checkpoint=False)


def prepare(batch_size=32, pin_memory=False, num_workers=0):
    """Reference main_no_ddp.py:22-34: the arguments are ignored; batch 64, reshuffled every epoch."""
    data, labels = load_dataset(_cfg)
    train_loader = DeviceLoader(data, labels, batch_size=_cfg.batch_size, device=device, sampler="random",
                                seed=_cfg.seed if _cfg.synthetic else None)
    print(len(train_loader))
    return train_loader


def training_loop(model, train_loader):
    """Reference main_no_ddp.py:36-59 (no checkpoint)."""
    from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
    kind = resolve_engine(_cfg, device, model) if isinstance(model, torch.nn.Module) else None
    if kind == "fused":
        n_idx = len(train_loader) * train_loader.batch_size
        # one process on a dedicated GPU: the automatic engine choice may give the sliced persistent engine the
        # whole device (batch 64 = 256 step workgroups, one per CU; with one CU kept free it would fall back to the
        # multi-kernel engine: 273.5 vs 97.9 us per step, profiles/bench_b64_r5f.log).  A batch above 64, or a
        # device with fewer CUs, still falls back to the multi-kernel engine with a warning.
        model = FusedDDPTrainer(model, train_loader.data, train_loader.labels, batch_max=train_loader.batch_size,
                                lr=_cfg.lr, dtype=_cfg.dtype, max_indices=max(n_idx, train_loader.batch_size),
                                full_device=True)
    elif kind == "ops":  # the ops-layer HIP kernels (flat parameters, packed weights, HIP SGD)
        from distributeddataparallel_cifar10_amd.ops.models import OpsModel
        from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP
        model = FlatBucketDDP(OpsModel(model, fp8=_cfg.fp8), bucket_cap_mb=_cfg.bucket_mb)
    try:
        return _train_loop(model, train_loader, 0, _cfg)
    finally:
        if hasattr(model, "close"):
            model.close()


if __name__ == "__main__":
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    add_cli_args(ap, batch_default=64)
    args = ap.parse_args()
    _cfg = config_from_args(args, data_path)
    _cfg.checkpoint = False
    print(f"Training on device {device}.")
    if _cfg.model == "resnet50":
        from distributeddataparallel_cifar10_amd.models.resnet50 import resnet50
        torch.manual_seed(_cfg.seed)
        model = resnet50(num_classes=10).to(device)
    else:
        model = NetResDeep().to(device)
    train_loader = prepare()
    training_loop(model, train_loader)
