"""NetResDeep: the weight-shared CIFAR-10 residual CNN of the reference.

Parity target: reference ``model/resnet.py:5-37``.

* ``NetResDeep(n_chans1=32, n_blocks=10)``: stem ``conv1`` (3->C, 3x3, pad 1, bias) -> ReLU -> 2x2 max-pool,
  a trunk that applies ONE ``ResBlock`` instance ``n_blocks`` times (``nn.Sequential(*(n_blocks * [blk]))``,
  reference ``model/resnet.py:10-11``), 2x2 max-pool, flatten (NCHW order), ``fc1`` (8*8*C -> 32) + ReLU,
  ``fc2`` (32 -> 10) logits.
* ``ResBlock(n_chans)``: conv (no bias) -> BatchNorm2d -> ReLU -> ``+ x`` (skip added AFTER the ReLU,
  reference ``model/resnet.py:33-37``), init kaiming_normal_(relu) / gamma 0.5 / beta 0
  (reference ``model/resnet.py:29-31``).

The weight sharing is load-bearing: 9 unique parameter tensors (76,074 params), 66 ``state_dict`` keys that alias
12 storages, and BN ``num_batches_tracked`` advancing by ``n_blocks`` per forward.

On the MI355X the training step of this module does NOT run through these torch ops: the fused engine in
``runtime/engine.py`` (HIP kernels in ``csrc/netresdeep_kernels.hip``) trains the very same parameter storage.
The torch forward below is the CPU path (``main_no_ddp.py`` on CPU) and the numerical oracle in ``tests/``.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F


class ResBlock(nn.Module):
    """conv3x3(no bias) -> BN -> ReLU -> + x   (reference ``model/resnet.py:24-37``)."""

    def __init__(self, n_chans: int):
        super().__init__()
        self.conv = nn.Conv2d(n_chans, n_chans, kernel_size=3, padding=1, bias=False)
        self.batch_norm = nn.BatchNorm2d(num_features=n_chans)
        torch.nn.init.kaiming_normal_(self.conv.weight, nonlinearity="relu")
        torch.nn.init.constant_(self.batch_norm.weight, 0.5)
        torch.nn.init.zeros_(self.batch_norm.bias)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = self.conv(x)
        out = self.batch_norm(out)
        out = torch.relu(out)
        return out + x


class NetResDeep(nn.Module):
    """Reference ``model/resnet.py:5-22`` with identical constructor, parameter names and state_dict."""

    def __init__(self, n_chans1: int = 32, n_blocks: int = 10):
        super().__init__()
        self.n_chans1 = n_chans1
        self.n_blocks = n_blocks
        self.conv1 = nn.Conv2d(3, n_chans1, kernel_size=3, padding=1)
        # ONE ResBlock instance repeated n_blocks times: shared conv weight and shared BN (reference :10-11).
        self.resblocks = nn.Sequential(*(n_blocks * [ResBlock(n_chans=n_chans1)]))
        self.fc1 = nn.Linear(8 * 8 * n_chans1, 32)
        self.fc2 = nn.Linear(32, 10)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        out = F.max_pool2d(torch.relu(self.conv1(x)), 2)
        out = self.resblocks(out)
        out = F.max_pool2d(out, 2)
        out = out.view(-1, 8 * 8 * self.n_chans1)
        out = torch.relu(self.fc1(out))
        out = self.fc2(out)
        return out

    # ---- helpers used by the fused engine / DDP wrapper -------------------------------------------------
    @property
    def block(self) -> ResBlock:
        """The single shared ResBlock instance."""
        return self.resblocks[0]

    def unique_named_parameters(self):
        """(name, param) for the 9 unique tensors, in registration order (shared block listed once)."""
        return list(self.named_parameters())  # named_parameters() already de-duplicates shared tensors
