"""Checkpointing with the reference's file format and without its write race.

Reference ``main.py:45``: ``torch.save(model.module.state_dict(), 'data/CIFAR-10/birds_vs_airplanes.pt')`` at
epochs 1, 10, ..., 90 from EVERY rank: a zip-format pickle of the un-prefixed OrderedDict
state_dict -- 66 keys aliasing 12 storages for NetResDeep -- last writer wins.

Here:
  * the same file name and the same state_dict (un-prefixed keys, fp32 tensors, aliasing kept, int64
    ``num_batches_tracked``), written by rank 0 only, atomically (tmp file + ``os.replace``);
  * the caller syncs BN buffers from rank 0 first (reference CC4 semantics), so the saved stats are rank 0's;
  * loading uses ``torch.load(weights_only=True)`` (never executes code from the file);
  * optional resume sidecar ``<path>.meta.json`` with epoch/step counters (an extension; the default file is
    unchanged).
"""
from __future__ import annotations

import json
import os
from typing import Optional

import torch
import torch.nn as nn

CHECKPOINT_NAME = "birds_vs_airplanes.pt"


def unwrap(model: nn.Module) -> nn.Module:
    """The innermost ``.module`` of DDP-style wrappers (FlatBucketDDP, ops.OpsModel, FusedDDPTrainer; reference
    main.py:45 strips the ``module.`` prefix the same way)."""
    while hasattr(model, "module") and isinstance(getattr(model, "module"), nn.Module):
        model = model.module
    return model


def export_state_dict(model: nn.Module) -> dict:
    """The reference-format state_dict: un-prefixed keys, tensors on the CPU (aliasing preserved)."""
    sd = unwrap(model).state_dict()
    cache = {}
    out = type(sd)()
    for k, v in sd.items():
        key = (v.untyped_storage().data_ptr(), v.storage_offset(), tuple(v.shape), tuple(v.stride()), v.dtype)
        if key not in cache:
            cache[key] = v.detach().to("cpu", copy=True)
        out[k] = cache[key]
    if hasattr(sd, "_metadata"):
        out._metadata = sd._metadata
    return out


def save_checkpoint(model: nn.Module, path: str, rank: int = 0, meta: Optional[dict] = None) -> Optional[str]:
    """Rank 0 writes `path` atomically; other ranks return None without touching the file."""
    if rank != 0:
        return None
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    sd = export_state_dict(model)
    tmp = f"{path}.tmp.{os.getpid()}"
    torch.save(sd, tmp)
    os.replace(tmp, path)
    if meta is not None:
        mtmp = f"{path}.meta.json.tmp.{os.getpid()}"
        with open(mtmp, "w") as f:
            json.dump(meta, f)
        os.replace(mtmp, f"{path}.meta.json")
    return path


def load_checkpoint(model: nn.Module, path: str, strict: bool = True, map_location="cpu") -> Optional[dict]:
    """Load a reference-format state_dict into `model` (weights_only).  Returns the resume sidecar if present."""
    sd = torch.load(path, map_location=map_location, weights_only=True)
    target = unwrap(model)
    with torch.no_grad():
        target.load_state_dict(sd, strict=strict)
    meta_path = f"{path}.meta.json"
    if os.path.exists(meta_path):
        with open(meta_path) as f:
            return json.load(f)
    return None
