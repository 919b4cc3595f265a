"""Logging / metrics: the reference's stdout lines plus optional JSON metrics.

Reference stdout, reproduced byte for byte by these helpers:
  ``main.py:82``      ``Using N GPUs``            (print("Using", n, "GPUs"))
  ``main.py:44``      ``Epoch {e}, Training loss {x}``   (rank-local mean over len(train_loader) batches)
  ``main.py:49``      ``training time: {s:.3f} seconds``
  ``main_no_ddp.py:20`` ``Training on device {device}.``
Extension: ``MetricsLog`` appends one JSON object per line (epoch, loss, step time, images/sec, rank).
"""
from __future__ import annotations

import json
import os
import time
from typing import Optional


def epoch_line(epoch: int, mean_loss: float) -> str:
    return "Epoch {}, Training loss {}".format(epoch, mean_loss)


def time_line(seconds: float) -> str:
    return f"training time: {seconds:.3f} seconds"


def should_log(epoch: int) -> bool:
    """Reference log/checkpoint cadence: epoch 1 and every 10th epoch (main.py:43)."""
    return epoch == 1 or epoch % 10 == 0


class MetricsLog:
    def __init__(self, path: Optional[str], rank: int = 0):
        self.path = path
        self.rank = rank
        if path:
            os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)

    def write(self, **rec) -> None:
        if not self.path:
            return
        rec.setdefault("rank", self.rank)
        rec.setdefault("time", time.time())
        with open(self.path, "a") as f:
            f.write(json.dumps(rec) + "\n")
