"""Index order of the reference's ``DistributedSampler`` (reference ``main.py:60``), as plain arrays.

``torch.utils.data.distributed.DistributedSampler(ds, num_replicas=W, rank=r)`` with its defaults
(shuffle=True, seed=0, drop_last=False):  ``randperm(N, generator=manual_seed(seed + epoch))``, padded by
wrapping to a multiple of W, then ``indices[rank::W]``.  The reference never calls ``set_epoch``,
so every epoch uses epoch 0's order; ``set_epoch=True`` here opts in to per-epoch reshuffling.

The engine consumes these indices on the device (no host DataLoader in the hot loop), so the order is computed
once per epoch as an int32 array.
"""
from __future__ import annotations

import math

import numpy as np
import torch


def distributed_indices(n: int, world_size: int = 1, rank: int = 0, seed: int = 0, epoch: int = 0,
                        shuffle: bool = True, drop_last: bool = False) -> np.ndarray:
    """Bit-identical to ``list(DistributedSampler(range(n), world_size, rank, shuffle, seed, drop_last))``."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside [0, {world_size})")
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        idx = torch.randperm(n, generator=g).numpy()
    else:
        idx = np.arange(n)
    if drop_last and n % world_size:
        num_samples = math.ceil((n - world_size) / world_size)
    else:
        num_samples = math.ceil(n / world_size)
    total = num_samples * world_size
    if not drop_last:
        pad = total - len(idx)
        if pad > 0:
            reps = math.ceil(pad / len(idx))
            idx = np.concatenate([idx] + [idx] * reps)[:total]
    else:
        idx = idx[:total]
    return np.ascontiguousarray(idx[rank:total:world_size].astype(np.int64))


def batches_per_epoch(n_local: int, batch: int, drop_last: bool = False) -> int:
    """``len(DataLoader(..., batch_size=batch, drop_last=drop_last))`` for `n_local` samples."""
    return n_local // batch if drop_last else -(-n_local // batch)
