"""Process-group bootstrap (reference ``main.py:21-24`` ``setup`` and ``main.py:65`` teardown).

The reference sets ``MASTER_ADDR=localhost``, ``MASTER_PORT=12355`` and calls
``init_process_group("nccl", rank, world_size)`` without binding a device.  Here:
  * backend ``"nccl"`` -- on ROCm this IS RCCL, over xGMI between the GPUs of the node;
  * the device is bound first (``torch.cuda.set_device(rank)``) and passed as ``device_id`` so the communicator is
    created eagerly on the right GPU;
  * MASTER_ADDR / MASTER_PORT already in the environment win (the reference's fixed port collides between
    concurrent jobs); the default address is 127.0.0.1 because the container hostname may not resolve;
  * ``gloo`` is accepted for CPU runs/tests; ``timeout_s`` sets the process-group timeout and
    ``TORCH_NCCL_ASYNC_ERROR_HANDLING=1`` makes a stuck collective raise (failure detection).
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

DEFAULT_PORT = 12355  # reference main.py:23


def setup(rank: int, world_size: int, backend: str = "nccl", port: Optional[int] = None,
          timeout_s: Optional[float] = None, local_rank: Optional[int] = None) -> None:
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    # a failed/timed-out RCCL collective aborts the communicator and raises instead of hanging (failure detection)
    os.environ.setdefault("TORCH_NCCL_ASYNC_ERROR_HANDLING", "1")
    if port is not None:
        os.environ["MASTER_PORT"] = str(port)
    else:
        os.environ.setdefault("MASTER_PORT", str(DEFAULT_PORT))
    kw = {}
    if timeout_s:
        kw["timeout"] = datetime.timedelta(seconds=float(timeout_s))
    if backend == "nccl":
        dev_idx = rank if local_rank is None else local_rank
        torch.cuda.set_device(dev_idx)
        kw["device_id"] = torch.device("cuda", dev_idx)
    dist.init_process_group(backend, rank=rank, world_size=world_size, **kw)


def teardown() -> None:
    if dist.is_available() and dist.is_initialized():
        dist.destroy_process_group()


def world() -> tuple[int, int]:
    """(rank, world_size); (0, 1) without a process group."""
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def params_checksum(module: torch.nn.Module) -> float:
    """Sum of all parameters (float64) -- cheap cross-rank consistency check."""
    with torch.no_grad():
        return float(sum(p.detach().double().sum().item() for p in module.parameters()))


def assert_params_in_sync(module: torch.nn.Module, atol: float = 0.0) -> None:
    """All ranks hold identical parameters (debug flag / tests)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    dev = next(module.parameters()).device
    c = torch.tensor([params_checksum(module)], dtype=torch.float64, device=dev)
    lo, hi = c.clone(), c.clone()
    dist.all_reduce(lo, op=dist.ReduceOp.MIN)
    dist.all_reduce(hi, op=dist.ReduceOp.MAX)
    if float(hi - lo) > atol:
        raise RuntimeError(f"parameters diverged across ranks: checksum spread {float(hi - lo):.3e}")
