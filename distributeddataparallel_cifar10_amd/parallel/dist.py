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


def device_key(dev) -> Optional[str]:
    """Identity of the physical device, to detect ranks that share one GPU: the device UUID, else the PCI
    domain:bus:device address; None when neither is known (then nobody is counted as sharing).  The local ordinal
    is never used: with one visible GPU per rank (HIP_VISIBLE_DEVICES) every rank is ``cuda:0``."""
    try:
        props = torch.cuda.get_device_properties(dev)
    except Exception:  # noqa: BLE001
        return None
    uuid = str(getattr(props, "uuid", "") or "")
    if uuid and uuid.strip("0-") != "":
        return "uuid:" + uuid
    bus = getattr(props, "pci_bus_id", None)
    if bus is not None and (bus or getattr(props, "pci_device_id", 0)):
        return f"pci:{getattr(props, 'pci_domain_id', 0)}:{bus}:{getattr(props, 'pci_device_id', 0)}"
    return None


def device_share_count(dev, group=None) -> int:
    """Collective: the largest number of ranks of `group` on one physical device (1 = one rank per GPU).  Unknown
    device identities count as unshared."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size(group) == 1:
        return 1
    keys = [None] * dist.get_world_size(group)
    dist.all_gather_object(keys, device_key(dev), group=group)
    known = [k for k in keys if k is not None]
    return max((known.count(k) for k in known), default=1)


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
