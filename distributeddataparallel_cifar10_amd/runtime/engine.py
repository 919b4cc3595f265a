"""Python face of the native NetResDeep training engine (``csrc/engine.hip``).

``NetResDeepEngine`` takes an ``nn.Module`` NetResDeep, re-homes its 9 unique parameters into ONE flat device
buffer (the module's ``nn.Parameter``s become views of it, so ``state_dict()`` / checkpoints always show what the
kernels train), and drives whole training steps that run as one hipGraph replay each.

Reference parity: the step is ``main.py:33-41`` (forward, CrossEntropyLoss, zero_grad, backward, SGD step,
``loss.item()`` accumulated) with DDP gradient averaging (``main.py:63``) when world_size > 1.  The loss is
accumulated on the device and read only at log points.
"""
from __future__ import annotations

import ctypes
import os
import warnings
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.nn as nn

from . import native

# ---- flat parameter layout (mirrors csrc/common.h) --------------------------------------------------------
FLAT_N = 76140
FLAT_ALLOC = 76160
OFF_RS = 76076
BUCKET_A_END = 65900
LAYOUT = {
    "fc1.weight": (0, (32, 2048)),
    "fc2.weight": (65536, (10, 32)),
    "fc1.bias": (65856, (32,)),
    "fc2.bias": (65888, (10,)),
    "resblocks.0.conv.weight": (65900, (32, 32, 3, 3)),
    "resblocks.0.batch_norm.weight": (75116, (32,)),
    "resblocks.0.batch_norm.bias": (75148, (32,)),
    "conv1.weight": (75180, (32, 3, 3, 3)),
    "conv1.bias": (76044, (32,)),
}
# engine kinds reported by dca_engine_kind (also written into bench / metrics output)
KIND_NAMES = {0: "multikernel", 2: "sliced"}
# gradient buckets (contiguous slices of the flat gradient buffer, ordered by gradient-ready time)
BUCKETS = (("fc", 0, BUCKET_A_END), ("trunk+stem+bn_stats", BUCKET_A_END, FLAT_N))


class _DcaInit(ctypes.Structure):
    _fields_ = [
        ("params", ctypes.c_void_p),
        ("grads", ctypes.c_void_p),
        ("rm", ctypes.c_void_p),
        ("rv", ctypes.c_void_p),
        ("nbt", ctypes.c_void_p),
        ("data", ctypes.c_void_p),
        ("labels", ctypes.c_void_p),
        ("n_data", ctypes.c_int),
        ("bmax", ctypes.c_int),
        ("bf16", ctypes.c_int),
        ("rows", ctypes.c_int),
        ("lr", ctypes.c_float),
        ("bn_mom", ctypes.c_float),
        ("bn_eps", ctypes.c_float),
        ("world_size", ctypes.c_int),
        ("rank", ctypes.c_int),
        ("nccl_id", ctypes.c_char_p),
        ("persistent", ctypes.c_int),
        ("debug", ctypes.c_int),
        ("pk_waves", ctypes.c_int),
        ("comm_mode", ctypes.c_int),
        ("force_comm", ctypes.c_int),
        ("auto_engine", ctypes.c_int),
        ("loopback", ctypes.c_int),
    ]


def bind_flat_parameters(model: nn.Module, device) -> tuple[torch.Tensor, torch.Tensor]:
    """Move NetResDeep's unique parameters into one flat buffer; params and grads become views of it."""
    flat = torch.zeros(FLAT_ALLOC, dtype=torch.float32, device=device)
    grads = torch.zeros(FLAT_ALLOC, dtype=torch.float32, device=device)
    names = dict(model.named_parameters())
    if set(names) != set(LAYOUT):
        raise ValueError(f"engine supports NetResDeep(32, 10) only; got parameters {sorted(names)}")
    for name, p in names.items():
        off, shape = LAYOUT[name]
        if tuple(p.shape) != shape:
            raise ValueError(f"{name}: expected shape {shape}, got {tuple(p.shape)}")
        n = p.numel()
        with torch.no_grad():
            flat[off:off + n].copy_(p.detach().reshape(-1))
        p.data = flat[off:off + n].view(shape)
        p.grad = grads[off:off + n].view(shape)
    return flat, grads


def tile_to_nhwc(raw: torch.Tensor, count: int, batch: int) -> torch.Tensor:
    """Fragment-tiled activations of the persistent engine -> NHWC [count, batch, 16, 16, 32].

    Tiled index of element (row, col = 4q + i, ch = 16h + c): row*512 + h*256 + (16q + c)*4 + i
    (csrc/netresdeep_pks.hip: st4r / ld4r)."""
    t = raw.reshape(count, batch, 16, 2, 4, 16, 4)  # [.., row, h, q, c, i]
    return t.permute(0, 1, 2, 4, 6, 3, 5).reshape(count, batch, 16, 16, 32)  # [.., row, q, i, h, c]


def nccl_unique_id() -> bytes:
    lib = native.require_native()
    buf = ctypes.create_string_buffer(128)
    native.check(lib.dca_nccl_unique_id(buf), "ncclGetUniqueId")
    return buf.raw


# The sliced engine's step epoch wraps here (csrc/netresdeep_pks.hip EPOCH_WRAP = 6 * 2^23).
EPOCH_WRAP = 6 << 23
S_SLICES = 4  # workgroups per image of the sliced step (csrc/netresdeep_pks.hip pks::S)


def coresident_budget(per_cu: int, ncu: int, n_share: int = 1, full_device: bool = False) -> int:
    """Spinning workgroups ONE rank may hold resident at once (csrc/engine.hip coresident_budget, same rule): the
    device's slots minus a margin -- one block per CU when several fit, else one CU (none only when a dedicated
    device was asked for explicitly) -- split evenly over the ranks sharing the device."""
    slots = per_cu * ncu
    margin = ncu if per_cu > 1 else (0 if full_device and n_share <= 1 else 1)
    return (slots - margin) // max(n_share, 1)


def max_sliced_batch(per_cu: int, ncu: int, n_share: int = 1, full_device: bool = False) -> int:
    """Largest per-rank batch whose sliced step (S_SLICES live workgroups per image) fits the budget."""
    return min(64, coresident_budget(per_cu, ncu, n_share, full_device) // S_SLICES)


@dataclass
class EngineConfig:
    batch_max: int = 32
    lr: float = 1e-2
    dtype: str = "bf16"          # "bf16": bf16 MFMA (fp32 accumulate/storage); "fp32": exact fp32 MFMA
    rows: int = 4                # multi-kernel engine: trunk rows per workgroup tile (2 or 4)
    persistent: Optional[bool] = None  # one-launch persistent step kernel (default: on; image-sliced)
    debug: bool = False          # persistent engine: also store per-block dy / residual grads (diagnostics)
    pk_waves: int = 8            # (ABI field; the sliced kernel always runs 8 waves per workgroup)
    world_size: int = 1
    rank: int = 0
    comm: str = "rccl"           # world_size > 1: "rccl" (all-reduce inside the graph-captured step),
                                 # "xgmi" (one-shot peer-to-peer all-reduce over IPC-mapped slabs, fused with
                                 # SGD; ranks of one node; call connect_peers() before stepping) or
                                 # "external" (host all-reduce between step parts; tests / any torch backend)
    bn_momentum: float = 0.1
    bn_eps: float = 1e-5
    force_comm: bool = False     # comm="rccl" at world_size 1: still run the graph-captured RCCL all-reduce and the
                                 # averaging SGD kernel (a 1-rank communicator) -- exercises that path on one GPU
    loopback: bool = False       # comm="xgmi" at world_size 1: the xGMI exchange with this rank as its own only peer
                                 # (uncached region, write-through slabs, flags, peer reads, averaging SGD): the
                                 # protocol's per-step cost measured on one device (bench.py --loopback)
    full_device: bool = False    # automatic engine choice on a device this process has to itself: the sliced step may
                                 # hold every CU (no slack CU), so batch 64 fits; a batch or a device that still does
                                 # not fit falls back to the multi-kernel engine (main_no_ddp.py)


class NetResDeepEngine:
    """Fused, graph-captured training step for NetResDeep on one MI355X (one rank of DDP)."""

    def __init__(self, model: nn.Module, data_u8: torch.Tensor, labels: torch.Tensor, cfg: EngineConfig,
                 nccl_id: Optional[bytes] = None, max_indices: Optional[int] = None):
        if cfg.comm not in ("rccl", "external", "xgmi"):
            raise ValueError("comm must be 'rccl', 'external' or 'xgmi'")
        if cfg.dtype not in ("bf16", "fp32"):
            raise ValueError("dtype must be 'bf16' or 'fp32'")
        auto_engine = cfg.persistent is None
        full_device = cfg.full_device or os.environ.get("DCA_PKS_ALLOW_FULL_DEVICE") == "1"
        if auto_engine:
            cfg.persistent = True  # the image-sliced persistent kernel (bf16 and fp32)
        if getattr(model, "n_chans1", 32) != 32 or getattr(model, "n_blocks", 10) != 10:
            raise ValueError("the fused engine is specialised for NetResDeep(n_chans1=32, n_blocks=10)")
        self.lib = native.require_native()
        dev = data_u8.device
        if dev.type != "cuda":
            raise ValueError("engine tensors must live on the GPU")
        self.cfg = cfg
        self.model = model
        self.device = dev
        assert data_u8.dtype == torch.uint8 and data_u8.dim() == 4 and tuple(data_u8.shape[1:]) == (3, 32, 32)
        self.data = data_u8.contiguous()
        self.labels = labels.to(device=dev, dtype=torch.int32).contiguous()
        self.flat, self.grads = bind_flat_parameters(model, dev)
        bn = model.resblocks[0].batch_norm
        self.bn = bn
        for name in ("running_mean", "running_var"):
            t = getattr(bn, name)
            if t.device != dev or not t.is_contiguous() or t.dtype != torch.float32:
                setattr(bn, name, t.to(dev, torch.float32).contiguous())
        if bn.num_batches_tracked.device != dev:
            bn.num_batches_tracked = bn.num_batches_tracked.to(dev)
        torch.cuda.synchronize(dev)
        self._nccl_id = ctypes.create_string_buffer(nccl_id or b"\0" * 128, 128)
        init = _DcaInit(
            params=self.flat.data_ptr(), grads=self.grads.data_ptr(),
            rm=bn.running_mean.data_ptr(), rv=bn.running_var.data_ptr(), nbt=bn.num_batches_tracked.data_ptr(),
            data=self.data.data_ptr(), labels=self.labels.data_ptr(), n_data=int(self.data.shape[0]),
            bmax=int(cfg.batch_max), bf16=1 if cfg.dtype == "bf16" else 0, rows=int(cfg.rows), lr=float(cfg.lr),
            bn_mom=float(cfg.bn_momentum), bn_eps=float(cfg.bn_eps), world_size=int(cfg.world_size),
            rank=int(cfg.rank), nccl_id=ctypes.cast(self._nccl_id, ctypes.c_char_p),
            persistent=1 if cfg.persistent else 0, debug=1 if cfg.debug else 0, pk_waves=int(cfg.pk_waves),
            comm_mode={"rccl": 0, "external": 1, "xgmi": 2}[cfg.comm], force_comm=1 if cfg.force_comm else 0,
            # the automatic choice keeps one CU of co-residency slack (batch 64 -> multi-kernel engine) unless the
            # caller owns the device (cfg.full_device, or DCA_PKS_ALLOW_FULL_DEVICE=1): then all 256 CUs
            auto_engine=1 if auto_engine and not full_device else 0,
            loopback=1 if cfg.loopback else 0,
        )
        self._init = init
        self.max_indices = int(max_indices or self.data.shape[0])
        h = ctypes.c_void_p()
        with torch.cuda.device(dev):
            rc = self.lib.dca_engine_create(ctypes.byref(init), self.max_indices, ctypes.byref(h))
            if rc != 0 and auto_engine and "cannot all be resident" in native.last_error():
                # the persistent step's workgroups do not fit the device at once (co-residency check at create
                # time): the multi-kernel engine instead, same numerics contract
                reason = native.last_error()
                cfg.persistent = False
                init.persistent = 0
                rc = self.lib.dca_engine_create(ctypes.byref(init), self.max_indices, ctypes.byref(h))
                warnings.warn(f"NetResDeepEngine: persistent step not co-resident ({reason}); using the multi-kernel "
                              f"engine (exact fp32 MFMA for dtype fp32, a different numerics path)", RuntimeWarning)
            native.check(rc, "dca_engine_create")
        self.h = h
        self.kind = int(self.lib.dca_engine_kind(h))  # 0 multi-kernel, 2 sliced persistent
        self.kind_name = KIND_NAMES.get(self.kind, str(self.kind))
        self.derive()
        self._n_indices = 0

    def set_shared_device(self, n: int) -> None:
        """Sliced engine, xGMI: ``n`` ranks share one device (shared-GPU rehearsal; the largest count over all
        devices, ``n <= 1``: not shared).  Then the reduction uses the coarse segment layout and the fc gradient
        segments run on the step kernel's fc workers only when every co-scheduled grid fits on the device
        (a rank's spinning kernels must always leave CUs for a peer's step).  Every rank must make the same
        call before stepping."""
        native.check(self.lib.dca_engine_set_shared_device(self.h, int(n)), "dca_engine_set_shared_device")

    def set_epoch(self, device_epoch: int, flag_epoch: int = 0) -> None:
        """Sliced engine: seed the step epoch and (xGMI) every exchange flag of this rank's region -- the epoch-wrap
        test hook (``EPOCH_WRAP - 3`` / ``2**32 - 3`` cross both wraps within a few steps).  xGMI: collective, every
        rank seeds the same values with no rank stepping (barrier before and after)."""
        flag = int(flag_epoch) & 0xFFFFFFFF
        flag = flag - (1 << 32) if flag >= (1 << 31) else flag  # the C int of the same bits
        native.check(self.lib.dca_engine_set_epoch(self.h, int(device_epoch), flag), "dca_engine_set_epoch")

    def epoch(self) -> int:
        """The device step epoch (synchronous)."""
        out = ctypes.c_int()
        native.check(self.lib.dca_engine_epoch(self.h, ctypes.byref(out)), "dca_engine_epoch")
        return int(out.value)

    def fc_in_step(self, batch: int) -> bool:
        """Whether a step at this batch size runs the fc gradient segments on the step kernel's fc workers."""
        return bool(self.lib.dca_engine_fc_in_step(self.h, int(batch)))

    def prologue(self, batch: int) -> bool:
        """Whether graph chunks at this batch size reduce each step's gradient segments in the next step's launch
        (DCA_PKS_PROLOGUE=1, where the budget and the all-reduce allow it)."""
        return bool(self.lib.dca_engine_prologue(self.h, int(batch)))

    # ---- state sync ---------------------------------------------------------------------------------------
    def derive(self):
        """Re-derive the kernel-layout weight copies after the fp32 params changed outside the engine."""
        torch.cuda.synchronize(self.device)
        native.check(self.lib.dca_engine_derive(self.h), "dca_engine_derive")

    def sync(self):
        native.check(self.lib.dca_engine_sync(self.h), "dca_engine_sync")

    # ---- xGMI peer mapping (comm="xgmi") --------------------------------------------------------------------
    def ipc_handle(self) -> bytes:
        """64-byte IPC handle of this rank's shared gradient region (to be all-gathered over the ranks)."""
        buf = ctypes.create_string_buffer(64)
        native.check(self.lib.dca_engine_ipc_handle(self.h, buf), "dca_engine_ipc_handle")
        return buf.raw

    def connect_peers(self, handles) -> None:
        """Map every rank's region (`handles`: world_size 64-byte handles in rank order)."""
        blob = b"".join(handles)
        if len(blob) != 64 * self.cfg.world_size:
            raise ValueError("need one 64-byte handle per rank")
        native.check(self.lib.dca_engine_ipc_open(self.h, blob, int(self.cfg.world_size)), "dca_engine_ipc_open")

    def xgmi_selftest(self, timeout_s: float = 20.0, rounds: int = 4) -> bool:
        """Collective: `rounds` consecutive all-reduces of rank- and round-dependent patterns through the xGMI
        protocol, each checked exactly.  Consecutive rounds alternate the slab parity and advance every
        workgroup's epoch, so a stale read of a previous round's slab (wrong parity, epoch reuse, a peer's L2
        holding an old line) shows up as a wrong sum.  Every rank must call it (it advances the shared epochs like
        a training step does)."""
        n, w, r = FLAT_N, self.cfg.world_size, self.cfg.rank
        base = torch.arange(n, device=self.device, dtype=torch.float32).remainder_(997.0)
        dst = torch.empty_like(base)
        ok = True
        for k in range(int(rounds)):
            # pattern_k(rank) = (rank + 1) * sign_k * (base + 7 k): integers, exact in fp32 after the sum
            sign = -1.0 if k % 2 else 1.0
            pat = (base + 7.0 * k) * sign
            src = pat * float(r + 1)
            dst.fill_(float("nan"))
            torch.cuda.synchronize(self.device)
            timed_out = ctypes.c_int()
            native.check(self.lib.dca_engine_ipc_selftest(self.h, src.data_ptr(), dst.data_ptr(), float(timeout_s),
                                                           ctypes.byref(timed_out)), "dca_engine_ipc_selftest")
            ok = ok and not timed_out.value and bool(torch.equal(dst, pat * float(w * (w + 1) // 2)))
            if self.cfg.persistent:  # the same exchange as the step kernel's fc workers run it (in-step bucket A)
                dst.fill_(float("nan"))
                torch.cuda.synchronize(self.device)
                lo, hi = ctypes.c_int(), ctypes.c_int()
                native.check(self.lib.dca_engine_ipc_selftest_fc(self.h, src.data_ptr(), dst.data_ptr(),
                                                                  float(timeout_s), ctypes.byref(timed_out),
                                                                  ctypes.byref(lo), ctypes.byref(hi)),
                             "dca_engine_ipc_selftest_fc")
                want = pat[lo.value:hi.value] * float(w * (w + 1) // 2)
                ok = ok and not timed_out.value and bool(torch.equal(dst[lo.value:hi.value], want))
        return ok

    def xgmi_bench(self, iters: int = 200) -> float:
        """Collective: mean microseconds per xGMI all-reduce of the flat gradient (protocol + data, no SGD)."""
        src = torch.ones(FLAT_N, device=self.device)
        dst = torch.empty_like(src)
        torch.cuda.synchronize(self.device)
        us = ctypes.c_float()
        native.check(self.lib.dca_engine_ipc_bench(self.h, src.data_ptr(), dst.data_ptr(), int(iters),
                                                   ctypes.byref(us)), "dca_engine_ipc_bench")
        self.check_errors()
        return float(us.value)

    # ---- data order -----------------------------------------------------------------------------------------
    def set_indices(self, indices) -> None:
        idx = np.ascontiguousarray(np.asarray(indices, dtype=np.int32))
        if idx.size and (idx.min() < 0 or idx.max() >= self.data.shape[0]):
            raise IndexError("sample index out of range")
        native.check(self.lib.dca_engine_set_indices(self.h, idx.ctypes.data, int(idx.size)), "set_indices")
        self._n_indices = int(idx.size)

    def set_cursor(self, pos: int = 0) -> None:
        native.check(self.lib.dca_engine_set_cursor(self.h, int(pos)), "set_cursor")

    # ---- stepping -------------------------------------------------------------------------------------------
    def run(self, batch: int, steps: int = 1, graph: bool = True) -> None:
        """Enqueue `steps` training steps of `batch` images each (asynchronous)."""
        native.check(self.lib.dca_engine_run(self.h, int(batch), int(steps), 1 if graph else 0), "dca_engine_run")

    def run_external(self, batch: int, steps: int, allreduce) -> None:
        """comm="external": `steps` steps whose gradient all-reduce is done by the host.  `allreduce(t)` must sum
        the fp32 device tensor `t` (the flat gradient buffer incl. the CC4 running-stat segment) over ranks in
        place, e.g. ``torch.distributed.all_reduce`` on any backend.  Synchronous, eager (no graph)."""
        if self.cfg.comm != "external" or self.cfg.world_size < 2:
            raise RuntimeError("run_external needs EngineConfig(comm='external', world_size > 1)")
        seg = self.grads[:FLAT_N]
        for _ in range(steps):
            native.check(self.lib.dca_engine_run_part(self.h, int(batch), 1), "run_part(1)")
            self.sync()
            allreduce(seg)
            torch.cuda.synchronize(self.device)
            native.check(self.lib.dca_engine_run_part(self.h, int(batch), 2), "run_part(2)")
        self.sync()

    def precapture(self, batch: int) -> None:
        """Capture the step graphs ``run(batch, ...)`` replays (16 / 8 / 4 / 2 / 1-step chunks) without running them, so
        a timed region never includes graph capture / instantiation."""
        native.check(self.lib.dca_engine_precapture(self.h, int(batch)), "dca_engine_precapture")

    def comm_time(self, reset: bool = False) -> tuple[float, int]:
        """(microseconds, calls) spent in the xGMI gradient all-reduce kernel (publish + wait for the slowest peer)
        since the last reset; (0.0, 0) on paths without it (world_size 1, RCCL).  Synchronises."""
        us, calls = ctypes.c_double(), ctypes.c_longlong()
        native.check(self.lib.dca_engine_comm_time(self.h, ctypes.byref(us), ctypes.byref(calls), int(reset)),
                     "dca_engine_comm_time")
        return float(us.value), int(calls.value)

    def check_errors(self, reset: bool = True) -> None:
        """Raise if a persistent-kernel BN exchange timed out (a workgroup was not co-resident)."""
        both = (ctypes.c_uint * 2)()
        native.check(self.lib.dca_engine_errors(self.h, both, int(reset)), "dca_engine_errors")
        flags = ctypes.c_uint(both[0])
        if both[1]:
            raise RuntimeError("xGMI gradient all-reduce: a peer's flag wait timed out (a rank stopped stepping?); "
                               "results of the affected steps are invalid")
        if flags.value:
            raise RuntimeError(f"persistent engine: BN-statistics exchange timed out (round mask {flags.value:#x}); "
                               "results of the affected steps are invalid")

    def read_loss(self, reset: bool = False) -> tuple[float, int]:
        """(sum of per-step mean losses, steps) since the last reset.  Synchronises."""
        self.check_errors()
        loss = ctypes.c_double()
        steps = ctypes.c_int()
        native.check(self.lib.dca_engine_read_loss(self.h, ctypes.byref(loss), ctypes.byref(steps), int(reset)),
                     "read_loss")
        return loss.value, steps.value

    def run_checked(self, batch: int, steps: int) -> int:
        """`steps` graph-replayed steps with the device error words checked after every 8-step chunk (pipelined:
        the GPU never waits for the check).  Synchronous.  Raises (``check_errors``) as soon as an exchange timed
        out -- a rank that stopped stepping is noticed within two chunks (< 16 steps), not at the epoch end.  Returns
        the steps run.  Only where every collective of the step is the engine's own (world size 1 or xGMI): a
        rank stopping early cannot leave its peers inside a graph-captured RCCL all-reduce, which has no deadline
        (``run_epoch`` uses plain replays there)."""
        done = ctypes.c_int()
        rc = self.lib.dca_engine_run_checked(self.h, int(batch), int(steps), ctypes.byref(done))
        if rc < 0:
            native.check(rc, "dca_engine_run_checked")
        if rc == 1:
            self.check_errors()  # raises (and resets the words)
            raise RuntimeError("engine error word set, but check_errors found none")
        return int(done.value)

    def run_epoch(self, indices, batch: int, graph: bool = True) -> tuple[float, int]:
        """One pass over `indices` in batches of `batch` (ragged last batch kept, drop_last=False).  With graphs at
        world size 1 or over xGMI the error words are checked after every chunk (``run_checked``); with RCCL every
        rank replays the whole epoch and the words are checked at its end (``read_loss``), so no rank stops
        stepping while its peers wait in a captured all-reduce."""
        n = len(indices)
        self.set_indices(indices)
        self.set_cursor(0)
        self.read_loss(reset=True)
        full, rem = divmod(n, batch)
        for b, k in ((batch, full), (rem, 1 if rem else 0)):
            if not k:
                continue
            if graph and (self.cfg.world_size == 1 or self.cfg.comm == "xgmi"):
                self.run_checked(b, k)
            else:
                self.run(b, k, graph)
        return self.read_loss(reset=True)

    # ---- introspection (tests) --------------------------------------------------------------------------
    def region(self, name: str, numel: int, dtype=torch.float32) -> torch.Tensor:
        """Copy of a workspace region (synchronises)."""
        self.sync()
        ptr = self.lib.dca_engine_region(self.h, name.encode())
        if not ptr:
            raise KeyError(name)
        out = torch.empty(numel, dtype=dtype, device=self.device)
        torch.cuda.synchronize(self.device)
        _copy_from_ptr(out, ptr)
        return out

    def activations(self, name: str, count: int, batch: int) -> torch.Tensor:
        """Per-block activation region (X, Y, DY, G) as NHWC [count, batch, 16, 16, 32].

        The multi-kernel engine stores NHWC directly.  The persistent engine stores the MFMA fragment-tiled layout
        [row][h][lane = 16q + c][i] holding element (row, col = 4q + i, ch = 16h + c) (netresdeep_pks.hip: st4r).
        """
        raw = self.region(name, count * batch * 8192)
        if not self.cfg.persistent:
            return raw.view(count, batch, 16, 16, 32)
        return tile_to_nhwc(raw, count, batch)

    def workspace_bytes(self) -> int:
        return int(self.lib.dca_engine_workspace_bytes(self.h))

    def close(self):
        if getattr(self, "h", None):
            self.lib.dca_engine_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _copy_from_ptr(out: torch.Tensor, ptr: int) -> None:
    """Copy out.numel() elements from raw device pointer `ptr` into `out` (same device)."""
    hip = _hip_runtime()
    nbytes = out.numel() * out.element_size()
    rc = hip.hipMemcpy(ctypes.c_void_p(out.data_ptr()), ctypes.c_void_p(ptr), ctypes.c_size_t(nbytes), 3)
    if rc != 0:
        raise RuntimeError(f"hipMemcpy failed: {rc}")


_HIP = None


def _hip_runtime():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so.7")
        _HIP.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        _HIP.hipMemcpy.restype = ctypes.c_int
    return _HIP
