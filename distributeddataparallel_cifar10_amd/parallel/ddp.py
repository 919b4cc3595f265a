"""Data-parallel training wrappers.

``FusedDDPTrainer`` is the MI355X fast path for NetResDeep: DDP semantics of reference ``main.py:63``
(``DistributedDataParallel(model, device_ids=[rank])``) implemented inside the native engine:

  * CC3 (construction): rank 0's parameters and BN buffers are broadcast to every rank;
  * CC5 (every backward): gradients averaged over ranks.  comm="xgmi" (default inside one node): a one-shot
    all-reduce in which every rank reads its peers' IPC-mapped gradient slabs directly over the xGMI links and
    applies SGD in the same kernel (csrc/xgmi_allreduce.hip); comm="rccl": flat RCCL all-reduce(s) captured in
    the step graph (bucket A = fc1/fc2 overlapped with the trunk backward in split mode);
  * CC4 (every forward): rank 0's BN running statistics reach every rank through a 64-float tail segment of
    the gradient buffer (no separate broadcast collective).

comm="auto" picks "xgmi" when every rank is on this node (LOCAL_WORLD_SIZE == WORLD_SIZE, or no launcher env)
and RCCL otherwise.  ``loopback=True`` (world size 1, comm="xgmi"): the xGMI exchange path runs with the rank as its
own only peer, so its per-step protocol cost is measurable on one device (``bench.py --allreduce xgmi --loopback``).  The xGMI path is verified at construction by a collective self-test (an exact all-reduce
of a known pattern); if mapping or the self-test fails on ANY rank, every rank falls back to RCCL together.

The generic ``FlatBucketDDP`` (any nn.Module, autograd hooks) lives in ``parallel/flat_ddp.py``.
"""
from __future__ import annotations

from typing import Optional

import os
import sys

import torch
import torch.distributed as dist
import torch.nn as nn

from ..runtime.engine import EngineConfig, NetResDeepEngine, nccl_unique_id
from .dist import device_share_count


def broadcast_module_state(model: nn.Module, src: int = 0) -> None:
    """CC3: make every rank's parameters and buffers equal to rank `src`'s (reference DDP constructor)."""
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return
    with torch.no_grad():
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, src)


class FusedDDPTrainer:
    """NetResDeep + DDP + SGD as one native, graph-captured training step per batch."""

    def __init__(self, model: nn.Module, data_u8: torch.Tensor, labels: torch.Tensor, batch_max: int = 32,
                 lr: float = 1e-2, dtype: str = "bf16", rows: int = 4, max_indices: Optional[int] = None,
                 persistent: Optional[bool] = None, comm: str = "auto", loopback: bool = False,
                 full_device: bool = False):
        world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        rank = dist.get_rank() if world > 1 else 0
        self.world_size, self.rank = world, rank
        if comm not in ("auto", "xgmi", "rccl"):
            raise ValueError("comm must be 'auto', 'xgmi' or 'rccl'")
        if comm == "auto":
            local = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
            comm = "xgmi" if 1 < world <= 8 and local == world else "rccl"
        args = dict(batch_max=batch_max, lr=lr, dtype=dtype, rows=rows, world_size=world, rank=rank,
                    persistent=persistent, full_device=full_device and world == 1)
        self.engine = None
        if loopback:
            if world != 1 or comm != "xgmi":
                raise ValueError("loopback needs world size 1 and comm='xgmi'")
            eng = NetResDeepEngine(model, data_u8, labels, EngineConfig(**args, comm="xgmi", loopback=True),
                                   max_indices=max_indices)
            if not eng.xgmi_selftest():
                eng.close()
                raise RuntimeError("xGMI loopback self-test failed")
            self.engine, self.comm, self.module, self.n_share = eng, "xgmi-loopback", model, 1
            return
        if world > 1:
            broadcast_module_state(model, 0)
        if world > 1 and comm == "xgmi":
            self.engine = self._try_xgmi(model, data_u8, labels, args, max_indices)
            if self.engine is None:
                comm = "rccl"
        if self.engine is None:
            nccl_id = None
            if world > 1:
                obj = [nccl_unique_id() if rank == 0 else None]
                dist.broadcast_object_list(obj, src=0)
                nccl_id = obj[0]
            cfg = EngineConfig(**args, comm="rccl")
            self.engine = NetResDeepEngine(model, data_u8, labels, cfg, nccl_id=nccl_id, max_indices=max_indices)
        self.comm = comm if world > 1 else "none"
        self.module = model

    def _try_xgmi(self, model, data_u8, labels, args, max_indices):
        """Create the engine with the xGMI all-reduce; None (on every rank) if any rank cannot use it."""
        eng, handle, err = None, None, None
        try:
            eng = NetResDeepEngine(model, data_u8, labels, EngineConfig(**args, comm="xgmi"), max_indices=max_indices)
            handle = eng.ipc_handle()
        except Exception as ex:  # noqa: BLE001 - any failure means: fall back on every rank
            err = ex
        handles = [None] * self.world_size
        dist.all_gather_object(handles, handle)
        ok = all(h is not None for h in handles)
        # ranks sharing one device (the shared-GPU rehearsal): a rank's spinning kernels (the step's fc workers,
        # the reduction) can hold CUs a peer's step needs -> the engine budgets its grids by the sharing count
        n_share = device_share_count(data_u8.device)
        self.n_share = n_share
        if ok and eng is not None and n_share > 1:
            eng.set_shared_device(n_share)
        if ok:
            try:
                eng.connect_peers(handles)
                ok = eng.xgmi_selftest()
                if not ok:
                    err = RuntimeError("self-test sum mismatch or timeout")
            except Exception as ex:  # noqa: BLE001
                ok, err = False, ex
        on_gpu = dist.get_backend() != "gloo"
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32, device=data_u8.device if on_gpu else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        if int(flag.item()) == 1:
            return eng
        if err is not None:
            print(f"[rank {self.rank}] xGMI all-reduce unavailable ({err}); using RCCL", file=sys.stderr)
        dist.barrier()  # every rank, so no peer still maps a region being freed
        if eng is not None:
            eng.close()
        return None

    def check_comm(self) -> None:
        """Raise if the engine recorded an exchange / all-reduce timeout (synchronous; called at epoch ends)."""
        if self.engine is not None:
            self.engine.check_errors()

    def close(self):
        if self.engine is None:
            return
        self.engine.sync()
        if self.world_size > 1:
            dist.barrier()  # no peer may still read this rank's shared region when it is freed
        self.engine.close()
        self.engine = None
