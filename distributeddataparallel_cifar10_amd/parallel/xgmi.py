"""Generic xGMI all-reduce communicator (``libdca_comm.so``, csrc/xgmi_comm.hip) for any model's flat buckets.

The reference's only collective is DDP's bucketed NCCL all-reduce (``main.py:63``, ``ppe_main_ddp.py:114``;
SURVEY.md 2.4 CC5).  Inside one MI355X node the 8 GPUs are fully connected by xGMI (7 point-to-point links per
GPU), so this communicator reads peers' buffers directly instead of running a ring:

* one-shot (small buckets): every rank reads the whole bucket from all peers at once and sums in rank order;
* two-shot (large buckets, e.g. ResNet-50): reduce-scatter by peer reads, then all-gather by peer reads --
  2(W-1)/W of the bucket per rank spread over all W-1 links (SURVEY.md 5.8 cost model).

Every rank exports one uncached region (``hipIpcGetMemHandle``); handles are all-gathered over the torch process
group (RCCL or gloo) and mapped with ``hipIpcOpenMemHandle``.  Calls are enqueued on a HIP stream with no host
synchronisation, so they overlap the backward on a comm stream and can be captured in a hipGraph.  A collective
self-test runs at construction; ``XgmiComm.create`` returns None on every rank if any rank cannot use the path
(the caller then falls back to the process group's all-reduce).
"""
from __future__ import annotations

import ctypes
import os
import sys
import threading
from typing import Optional

import torch
import torch.distributed as dist

from .. import build as _build
from .dist import device_share_count

ABI_VERSION = 1
_lock = threading.Lock()
_lib = None
ALGOS = {"auto": 0, "oneshot": 1, "twoshot": 2}


def lib():
    """The loaded comm library (built first if the sources changed); raises if it cannot be loaded."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = _build.lib_path("comm")
        try:
            path = _build.build(variant="comm")
        except Exception as exc:  # toolchain missing: only acceptable if the .so already exists
            if not os.path.exists(path):
                raise RuntimeError(f"cannot build the comm library: {exc}") from exc
        L = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        vp, ci, cll, cf = ctypes.c_void_p, ctypes.c_int, ctypes.c_longlong, ctypes.c_float
        L.dca_comm_last_error.restype = ctypes.c_char_p
        L.dca_comm_flag_bytes.restype = cll
        L.dca_comm_create.argtypes = [ci, ci, cll, ci, ctypes.POINTER(vp)]
        L.dca_comm_ipc_handle.argtypes = [vp, ctypes.c_char_p]
        L.dca_comm_open.argtypes = [vp, ctypes.c_char_p]
        L.dca_comm_allreduce.argtypes = [vp, vp, vp, cll, ci, ci, cf, cf, vp, ctypes.POINTER(ci)]
        L.dca_comm_errors.argtypes = [vp, ctypes.POINTER(ctypes.c_uint), ci]
        L.dca_comm_destroy.argtypes = [vp]
        if L.dca_comm_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: ABI {L.dca_comm_abi_version()} != {ABI_VERSION} (stale build?)")
        _lib = L
        return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"xgmi {what} failed: {lib().dca_comm_last_error().decode(errors='replace')}")


class XgmiComm:
    """One rank's endpoint.  ``all_reduce_(t)`` sums (``average=True``: averages) a contiguous fp32 CUDA tensor
    of at most ``max_numel`` elements across the group, in place, on ``stream`` (default: current stream)."""

    def __init__(self, max_numel: int, group=None, wire: str = "fp32", nb: Optional[int] = 128,
                 timeout_s: float = 30.0):
        if wire not in ("fp32", "bf16"):
            raise ValueError("wire must be 'fp32' or 'bf16'")
        self.group = group
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.world > 8:
            raise ValueError("the xGMI communicator spans one node (<= 8 ranks)")
        self.wire, self.timeout_s, self.max_numel = wire, float(timeout_s), int(max_numel)
        nb = 128 if nb is None else int(nb)
        self.nb = nb
        self.last_algo = None
        # auto choice between one-shot and two-shot: the library's modelled crossover until calibrate() measured
        # this node's own (bytes on the wire: one-shot below, two-shot from there)
        self.crossover_bytes: Optional[int] = None
        self.calibration = None
        h = ctypes.c_void_p()
        slab = (self.max_numel + 3) // 4 * 4 * 4  # fp32 sized, so the wire format can be switched per call
        _check(lib().dca_comm_create(self.rank, self.world, slab, int(nb), ctypes.byref(h)), "create")
        self._h = h

    # ---- collective setup -------------------------------------------------------------------------------------
    def handle(self) -> bytes:
        buf = ctypes.create_string_buffer(64)
        _check(lib().dca_comm_ipc_handle(self._h, buf), "ipc_handle")
        return buf.raw

    def connect(self, handles) -> None:
        if self.world > 1:
            _check(lib().dca_comm_open(self._h, b"".join(handles)), "open")

    @classmethod
    def create(cls, max_numel: int, group=None, device=None, verbose: bool = True, **kw) -> Optional["XgmiComm"]:
        """Collective: build, connect and self-test the communicator on every rank; None on EVERY rank if any
        rank failed (so all ranks agree on the fallback)."""
        world = dist.get_world_size(group) if dist.is_initialized() else 1
        if kw.get("nb") is None:
            # ranks sharing one device (the shared-GPU rehearsal): every rank's call spins until all have arrived,
            # so the W grids must be co-resident together -- split the default 128 workgroups by the sharing count
            kw["nb"] = max(8, 128 // device_share_count(device, group))
        comm, handle, err = None, None, None
        try:
            comm = cls(max_numel, group=group, **kw)
            handle = comm.handle()
        except Exception as ex:  # noqa: BLE001 - any failure means: fall back on every rank
            err = ex
        handles = [None] * world
        if world > 1:
            dist.all_gather_object(handles, handle, group=group)
        else:
            handles = [handle]
        ok = all(h is not None for h in handles)
        if ok:
            try:
                comm.connect(handles)
                ok = comm.self_test(device)
                if not ok:
                    err = RuntimeError("self-test sum mismatch or timeout")
            except Exception as ex:  # noqa: BLE001
                ok, err = False, ex
        if world > 1:
            flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                                device="cpu" if dist.get_backend(group) == "gloo" else device)
            dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
            ok = int(flag.item()) == 1
        if ok and world > 2 and os.environ.get("DCA_XGMI_CALIBRATE", "1") != "0":
            comm.calibrate(device)
        if ok:
            return comm
        if err is not None and verbose:
            print(f"[rank {dist.get_rank(group) if dist.is_initialized() else 0}] xGMI communicator unavailable "
                  f"({err}); using the process group's all-reduce", file=sys.stderr)
        if world > 1:
            dist.barrier(group=group)  # no peer may still map a region being freed
        if comm is not None:
            comm.close(barrier=False)
        return None

    def self_test(self, device=None) -> bool:
        """Every rank contributes (rank + 1) * ramp; both algorithms and both wire formats must give the exact
        analytic sum (small integers: exact in bf16 too) on every rank, within the timeout."""
        n = min(self.max_numel, 65536 + 3)  # odd size: exercises the partial last float4
        ramp = torch.arange(n, device=device, dtype=torch.float32).remainder_(13.0)  # inputs <= 96: exact in bf16
        expect = ramp * (self.world * (self.world + 1) / 2)
        good = True
        for algo in ("oneshot", "twoshot"):
            for wire in ("fp32", "bf16"):
                t = ramp * float(self.rank + 1)
                self.all_reduce_(t, average=False, algo=algo, wire=wire)
                ref = expect.to(torch.bfloat16).float() if wire == "bf16" else expect  # one final RNE rounding
                good &= bool(torch.equal(t, ref))
        return good and self.errors() == 0

    def calibrate(self, device=None, reps: int = 5) -> Optional[int]:
        """Collective: measure the one-shot / two-shot crossover on this node instead of trusting the library's
        model (L = 5 us per flag round trip, B = 350 GB/s per GPU; comm_api.hip).  Every rank times both algorithms
        on the same bucket sizes (64 KiB x 4^k up to the slab, on the comm's wire format); the per-size time is the
        MAX over ranks (one all-reduce of the timing vector), so every rank derives the same crossover: the smallest
        size from which two-shot wins at every larger measured size too.  W <= 2: one-shot always moves no more
        bytes, nothing to measure."""
        if self.world <= 2:
            return None
        wire_b = 2 if self.wire == "bf16" else 4
        sizes, n = [], 16384
        while n <= self.max_numel:
            sizes.append(n)
            n *= 4
        if not sizes:
            return None
        buf = torch.zeros(sizes[-1], device=device, dtype=torch.float32)
        st = torch.cuda.current_stream(buf.device)
        times = []
        for n in sizes:
            t = buf[:n]
            for algo in ("oneshot", "twoshot"):
                for _ in range(2):
                    self.all_reduce_(t, average=False, algo=algo)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record(st)
                for _ in range(reps):
                    self.all_reduce_(t, average=False, algo=algo)
                e1.record(st)
                e1.synchronize()
                times.append(e0.elapsed_time(e1) * 1e3 / reps)  # us per call
        if self.errors(reset=False):  # a peer wait expired: no timing is trusted (and check() will still report it)
            times = [float("inf")] * len(times)
        # every rank reaches this all-reduce, failed or not, so no rank is left waiting in it
        tv = torch.tensor(times, dtype=torch.float64,
                          device="cpu" if dist.get_backend(self.group) == "gloo" else buf.device)
        dist.all_reduce(tv, op=dist.ReduceOp.MAX, group=self.group)
        tv = tv.cpu().tolist()
        if any(v == float("inf") for v in tv):
            self.calibration = {"failed": True, "world": self.world}
            return None  # the library's modelled crossover stays in use
        one, two = tv[0::2], tv[1::2]
        cross = self.pick_crossover([n * wire_b for n in sizes], one, two)
        self.crossover_bytes = cross if cross is not None else (1 << 62)  # never: one-shot everywhere measured
        self.calibration = {"bytes": [n * wire_b for n in sizes], "oneshot_us": one, "twoshot_us": two,
                            "crossover_bytes": cross, "world": self.world}
        return cross

    @staticmethod
    def pick_crossover(sizes_bytes, oneshot_us, twoshot_us) -> Optional[int]:
        """The smallest measured size from which two-shot is faster at that size and every larger one (None: it
        never is).  A two-shot win at a small size followed by a loss above it is noise, not a crossover."""
        cross = None
        for i in range(len(sizes_bytes) - 1, -1, -1):  # walk down while two-shot keeps winning
            if twoshot_us[i] < oneshot_us[i]:
                cross = int(sizes_bytes[i])
            else:
                break
        return cross

    # ---- the collective ---------------------------------------------------------------------------------------
    def all_reduce_(self, t: torch.Tensor, average: bool = True, algo: str = "auto", wire: Optional[str] = None,
                    stream: Optional[torch.cuda.Stream] = None) -> torch.Tensor:
        if t.dtype != torch.float32 or not t.is_cuda or not t.is_contiguous():
            raise ValueError("xGMI all-reduce takes a contiguous fp32 CUDA tensor")
        if t.numel() > self.max_numel:
            raise ValueError(f"tensor of {t.numel()} elements exceeds the communicator's {self.max_numel}")
        if t.data_ptr() % 16:
            raise ValueError("xGMI all-reduce needs a 16-byte aligned tensor")
        st = stream if stream is not None else torch.cuda.current_stream(t.device)
        if algo == "auto" and self.crossover_bytes is not None:  # the measured crossover (calibrate())
            algo = "twoshot" if t.numel() * (2 if (wire or self.wire) == "bf16" else 4) >= self.crossover_bytes \
                else "oneshot"
        used = ctypes.c_int()
        _check(lib().dca_comm_allreduce(self._h, ctypes.c_void_p(t.data_ptr()), ctypes.c_void_p(t.data_ptr()),
                                        t.numel(), 1 if (wire or self.wire) == "bf16" else 0, ALGOS[algo],
                                        1.0 / self.world if average else 1.0, self.timeout_s,
                                        ctypes.c_void_p(st.cuda_stream), ctypes.byref(used)), "allreduce")
        self.last_algo = {1: "oneshot", 2: "twoshot"}[used.value]
        return t

    def errors(self, reset: bool = True) -> int:
        """Synchronous: the device error word (bit 0 = a peer flag wait expired)."""
        out = ctypes.c_uint()
        _check(lib().dca_comm_errors(self._h, ctypes.byref(out), 1 if reset else 0), "errors")
        return int(out.value)

    def check(self) -> None:
        e = self.errors()
        if e:
            raise RuntimeError(f"xGMI all-reduce: a peer did not arrive within {self.timeout_s} s (error 0x{e:x})")

    def close(self, barrier: bool = True) -> None:
        if getattr(self, "_h", None) is None:
            return
        torch.cuda.synchronize()
        if barrier and self.world > 1 and dist.is_initialized():
            dist.barrier(group=self.group)  # no peer may still read this rank's region when it is freed
        lib().dca_comm_destroy(self._h)
        self._h = None
