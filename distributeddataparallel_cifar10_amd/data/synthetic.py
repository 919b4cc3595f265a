"""Synthetic CIFAR-10-shaped data (no network: the real dataset cannot be downloaded here).

Same shapes/dtypes as the CIFAR-10 train split read by reference ``main.py:53``: 50,000 uint8 images 3x32x32
(CHW, as stored in the CIFAR python batches) and int64 labels in [0, 10).  Deterministic for a given seed, so
every rank of a DDP job sees the same dataset (as every rank of the reference reads the same files).
"""
from __future__ import annotations

import torch


def synthetic_cifar(n: int = 50000, seed: int = 0, num_classes: int = 10):
    g = torch.Generator().manual_seed(seed)
    data = torch.randint(0, 256, (n, 3, 32, 32), dtype=torch.uint8, generator=g)
    labels = torch.randint(0, num_classes, (n,), dtype=torch.int64, generator=g)
    return data, labels
