"""Device-resident batch loader: the MI355X replacement of the reference's host DataLoader.

Reference ``main.py:60-61``: ``DataLoader(cifar10, batch_size=32, drop_last=False, shuffle=False,
sampler=DistributedSampler(cifar10, num_replicas=W, rank=r))`` with ``num_workers=0`` -- every step decodes 32 PIL
images on the host and copies them to the GPU (<= ~20k img/s per rank).  Reference
``main_no_ddp.py:31``: ``DataLoader(cifar10, batch_size=64, shuffle=True)`` (a fresh random order every epoch).

Here the uint8 dataset (150 MB for CIFAR-10) is uploaded to HBM once.  An epoch is an index array
(``data/sampler.py``); the fused engine gathers + normalises a batch inside its stem kernel, and the generic torch
path (``__iter__``) gathers + normalises on the device.  ``len(loader)`` equals the reference DataLoader's length
(ragged last batch kept), which is what the printed mean loss divides by (``main.py:44``).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .cifar import normalize_u8
from .sampler import batches_per_epoch, distributed_indices


class DeviceLoader:
    def __init__(self, data_u8: torch.Tensor, labels: torch.Tensor, batch_size: int = 32, world_size: int = 1,
                 rank: int = 0, device=None, sampler: str = "distributed", seed: Optional[int] = 0, drop_last: bool = False,
                 set_epoch: bool = False):
        if sampler not in ("distributed", "random", "sequential"):
            raise ValueError("sampler must be 'distributed', 'random' or 'sequential'")
        device = torch.device(device) if device is not None else data_u8.device
        self.data = data_u8.to(device).contiguous()
        self.labels = labels.to(device=device, dtype=torch.int64).contiguous()
        self.batch_size = int(batch_size)
        self.world_size, self.rank = int(world_size), int(rank)
        self.sampler, self.drop_last, self.reshuffle = sampler, bool(drop_last), set_epoch
        self.seed = int(seed) if seed is not None else 0
        self.device = device
        self.epoch = 0
        self._random_gen = np.random.default_rng(seed if sampler == "random" else None)

    @property
    def n(self) -> int:
        return int(self.data.shape[0])

    def set_epoch(self, epoch: int) -> None:
        """Select the epoch's order (honoured for 'distributed' only if constructed with set_epoch=True, as the
        reference never calls DistributedSampler.set_epoch)."""
        self.epoch = int(epoch)

    def indices(self) -> np.ndarray:
        """This rank's sample order for the current epoch."""
        if self.sampler == "distributed":
            return distributed_indices(self.n, self.world_size, self.rank, seed=self.seed,
                                       epoch=self.epoch if self.reshuffle else 0, drop_last=self.drop_last)
        if self.sampler == "random":  # RandomSampler: a new permutation on every pass
            return self._random_gen.permutation(self.n).astype(np.int64)
        return np.arange(self.n, dtype=np.int64)

    def __len__(self) -> int:
        n_local = len(distributed_indices(self.n, self.world_size, self.rank, shuffle=False,
                                          drop_last=self.drop_last)) if self.sampler == "distributed" else self.n
        return batches_per_epoch(n_local, self.batch_size, self.drop_last)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        idx = torch.from_numpy(self.indices()).to(self.device)
        for s in range(0, len(idx), self.batch_size):
            b = idx[s:s + self.batch_size]
            if self.drop_last and len(b) < self.batch_size:
                break
            yield normalize_u8(self.data.index_select(0, b)), self.labels.index_select(0, b)


def make_loader(data_u8: torch.Tensor, labels: torch.Tensor, batch_size: int, world_size: int = 1, rank: int = 0,
                device: Optional[torch.device] = None, **kw) -> DeviceLoader:
    return DeviceLoader(data_u8, labels, batch_size, world_size, rank, device, **kw)
