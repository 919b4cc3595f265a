"""Practical-bar measurement: the reference's training step run AS-IS with stock PyTorch-ROCm eager ops.

This is NOT our framework: it reproduces reference ``main.py:26-41`` (SGD 1e-2, CrossEntropy, ``loss.item()`` every
step, stock ``torch.nn.parallel.DistributedDataParallel`` at world_size 1 over RCCL) on the reference model, so the
speedup of the fused engine can be quoted against the same hardware.

Two data modes:
  * ``--data host``: per-sample host pipeline like torchvision's CIFAR10 + ToTensor + Normalize + default collate
    (reference ``main.py:53-61``; torchvision is absent here, so the transform is emulated with torch ops on
    uint8 HWC arrays, which is what torchvision does after PIL decode).
  * ``--data device``: batches pre-staged on the GPU (isolates the eager step cost).

Prints one JSON line per mode.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch
import torch.distributed as dist
import torch.nn as nn
import torch.optim as optim

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model.resnet import NetResDeep  # noqa: E402

MEAN = torch.tensor([0.4915, 0.4823, 0.4468]).view(3, 1, 1)
STD = torch.tensor([0.2470, 0.2435, 0.2616]).view(3, 1, 1)


class FakeCifar(torch.utils.data.Dataset):
    def __init__(self, n=50000):
        g = torch.Generator().manual_seed(0)
        self.data = torch.randint(0, 256, (n, 32, 32, 3), dtype=torch.uint8, generator=g).numpy()
        self.targets = torch.randint(0, 10, (n,), generator=g).tolist()

    def __len__(self):
        return len(self.targets)

    def __getitem__(self, i):
        img = torch.from_numpy(self.data[i]).permute(2, 0, 1).float().div_(255.0)  # ToTensor
        img = (img - MEAN) / STD  # Normalize
        return img, self.targets[i]


def run(mode: str, steps: int, warmup: int, bs: int, dtype: str = "fp32") -> dict:
    dev = torch.device("cuda", 0)
    model = NetResDeep().to(dev)
    model = nn.parallel.DistributedDataParallel(model, device_ids=[0], output_device=0)
    opt = optim.SGD(model.parameters(), lr=1e-2)
    loss_fn = nn.CrossEntropyLoss()
    if mode == "host":
        ds = FakeCifar()
        sampler = torch.utils.data.distributed.DistributedSampler(ds, num_replicas=1, rank=0)
        loader = torch.utils.data.DataLoader(ds, batch_size=bs, drop_last=False, shuffle=False, sampler=sampler)
        it = iter(loader)

        def nxt():
            nonlocal it
            try:
                return next(it)
            except StopIteration:
                it = iter(loader)
                return next(it)
    else:
        xs = torch.randn(8, bs, 3, 32, 32, device=dev)
        ys = torch.randint(0, 10, (8, bs), device=dev)
        k = [0]

        def nxt():
            k[0] += 1
            return xs[k[0] % 8], ys[k[0] % 8]

    def step():
        imgs, labels = nxt()
        imgs, labels = imgs.to(dev), labels.to(dev)
        with torch.autocast("cuda", torch.bfloat16, enabled=dtype == "bf16"):  # bf16: AMP, fp32 master weights
            out = model(imgs)
            loss = loss_fn(out.float(), labels)
        opt.zero_grad()
        loss.backward()
        opt.step()
        return loss.item()

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"metric": "reference_eager_images_per_sec", "data": mode, "value": steps * bs / dt,
            "ms_per_step": 1e3 * dt / steps, "steps": steps, "batch": bs, "n_gpus": 1, "dtype": dtype}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=30)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--modes", default="device,host")
    ap.add_argument("--dtypes", default="fp32", help="comma list of fp32 / bf16 (torch.autocast bf16)")
    a = ap.parse_args()
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    dist.init_process_group("nccl", rank=0, world_size=1)
    torch.cuda.set_device(0)
    for d in a.dtypes.split(","):
        for m in a.modes.split(","):
            print(json.dumps(run(m, a.steps, a.warmup, a.batch, d)), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
