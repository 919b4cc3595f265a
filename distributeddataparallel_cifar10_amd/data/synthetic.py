"""Synthetic CIFAR-10-shaped data (no network: the real dataset cannot be downloaded here).

Same shapes/dtypes as the CIFAR-10 train split read by reference ``main.py:53``: 50,000 uint8 images 3x32x32
(CHW, as stored in the CIFAR python batches) and int64 labels in [0, 10).  Deterministic for a given seed, so
every rank of a DDP job sees the same dataset (as every rank of the reference reads the same files).

``learnable=True`` (``"easy"``): the label is a function of the image -- every image of class c is that class's
colour (a fixed palette of 10 well-separated RGB triples) plus a class-specific stripe pattern and uniform pixel noise
-- so a run shows a falling loss (the random-label default stays at ln 10 = 2.3026 for ever, which says nothing about
learning; reference ``main.py:43-44`` prints exactly this loss).  It is nearly trivial: the colour alone separates
the classes, and the epoch-1 mean loss of a full run is ~0.03.

``learnable="hard"`` (the CLI's ``--synthetic-learnable``): a task with a learning curve.
  * colour: the class palette entry blended 50/50 with a per-image random colour, so the colour clusters of
    neighbouring classes overlap;
  * stripes: the class's period (2 .. 6 px) and orientation, at a random per-image phase, amplitude 24 under
    +-64 pixel noise (the texture, not the colour, is what separates the classes reliably);
  * 10 % label noise: the label of a random tenth of the images is redrawn uniformly (images keep their true class's
    pattern), so the loss has an irreducible floor near 0.5 (CE of a perfect classifier: -(0.91 ln 0.91 + 0.09
    ln 0.01) = 0.50) until the network starts to memorise the flipped labels.
"""
from __future__ import annotations

import torch

# 10 distinct colours (uint8 RGB), pairwise >= 80 apart in at least one channel
_PALETTE = [(200, 60, 60), (60, 200, 60), (60, 60, 200), (200, 200, 60), (200, 60, 200),
            (60, 200, 200), (130, 130, 130), (230, 150, 40), (40, 110, 170), (150, 40, 110)]


def synthetic_cifar(n: int = 50000, seed: int = 0, num_classes: int = 10, learnable=False):
    g = torch.Generator().manual_seed(seed)
    if learnable == "hard":
        return _hard(n, g, num_classes)
    if learnable not in (False, True, "easy"):
        raise ValueError(f"learnable must be False, True / 'easy' or 'hard' (got {learnable!r})")
    if not learnable:
        data = torch.randint(0, 256, (n, 3, 32, 32), dtype=torch.uint8, generator=g)
        labels = torch.randint(0, num_classes, (n,), dtype=torch.int64, generator=g)
        return data, labels
    if num_classes > len(_PALETTE):
        raise ValueError(f"learnable synthetic data has {len(_PALETTE)} classes")
    labels = torch.randint(0, num_classes, (n,), dtype=torch.int64, generator=g)
    colour = torch.tensor(_PALETTE, dtype=torch.int16)[labels]                    # [n, 3]
    # class c: stripes of period 2 + c // 2 pixels, horizontal for even c, vertical for odd c, amplitude 30
    pos = torch.arange(32, dtype=torch.int16)
    period = (2 + labels // 2).to(torch.int16)                                    # [n]
    phase = (pos[None, :] // period[:, None]) % 2                                 # [n, 32]
    horiz = (labels % 2 == 0)[:, None, None]
    stripe = torch.where(horiz, phase[:, :, None].expand(n, 32, 32), phase[:, None, :].expand(n, 32, 32))
    noise = torch.randint(-48, 49, (n, 3, 32, 32), dtype=torch.int16, generator=g)
    img = colour[:, :, None, None] + 30 * stripe[:, None].to(torch.int16) - 15 + noise
    return img.clamp_(0, 255).to(torch.uint8), labels


def _hard(n: int, g: torch.Generator, num_classes: int):
    if num_classes > len(_PALETTE):
        raise ValueError(f"learnable synthetic data has {len(_PALETTE)} classes")
    true = torch.randint(0, num_classes, (n,), dtype=torch.int64, generator=g)
    mix = torch.randint(0, 256, (n, 3), dtype=torch.int16, generator=g)
    colour = (torch.tensor(_PALETTE, dtype=torch.int16)[true] + mix) // 2                 # [n, 3]
    pos = torch.arange(32, dtype=torch.int16)
    period = (2 + true // 2).to(torch.int16)                                              # [n]
    shift = torch.randint(0, 64, (n,), dtype=torch.int16, generator=g) % period           # random phase
    phase = ((pos[None, :] + shift[:, None]) // period[:, None]) % 2                     # [n, 32]
    horiz = (true % 2 == 0)[:, None, None]
    stripe = torch.where(horiz, phase[:, :, None].expand(n, 32, 32), phase[:, None, :].expand(n, 32, 32))
    noise = torch.randint(-64, 65, (n, 3, 32, 32), dtype=torch.int16, generator=g)
    img = colour[:, :, None, None] + 24 * stripe[:, None].to(torch.int16) - 12 + noise
    flip = torch.rand(n, generator=g) < 0.1
    labels = torch.where(flip, torch.randint(0, num_classes, (n,), dtype=torch.int64, generator=g), true)
    return img.clamp_(0, 255).to(torch.uint8), labels
