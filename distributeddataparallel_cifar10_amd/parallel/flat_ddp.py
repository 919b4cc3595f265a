"""Generic flat-bucket data parallelism for any ``nn.Module`` (the stock-op path of the framework).

Reference: ``DDP(model, device_ids=[rank], output_device=rank)`` (``main.py:63``), whose implicit behaviour is
pinned down in SURVEY.md section 2.4:
  * CC3 -- at construction rank 0's parameters and buffers are broadcast to every rank;
  * CC4 -- at every forward rank 0's buffers (BN running stats, num_batches_tracked) are broadcast
    (``broadcast_buffers=True``);
  * CC5 -- during backward, gradients are averaged over ranks bucket by bucket.

Design (not a copy of the c10d Reducer):
  * all unique parameters live in ONE flat buffer and all gradients in ONE flat gradient buffer; ``p.data`` /
    ``p.grad`` are views, so there is no bucket copy-in/copy-out and the SGD update is one fused op over the flat
    buffer (``FlatSGD``);
  * the flat layout is REVERSE registration order (approximately gradient-ready order), so every bucket is a
    contiguous slice that becomes ready as a unit;
  * a bucket's all-reduce is launched asynchronously from the gradient hook of its last parameter, so it
    overlaps the rest of the backward (RCCL runs on its own HIP stream); the backward's final callback waits
    for all buckets;
  * bucket sizes default to a cap sized for xGMI (``bucket_cap_mb``): big enough that a ring step moves well over
    64 KB per link, small enough that the first bucket fires early.  With ``first_bucket_mb`` the first (earliest
    ready) bucket can be made smaller, like DDP's 1 MiB first bucket.

  * the bucket all-reduce is either the process group's (RCCL over xGMI on GPUs, gloo on CPU) or, for CUDA
    models inside one node, the framework's own xGMI peer-read all-reduce (``parallel/xgmi.py``: one-shot for
    small buckets, two-shot reduce-scatter/all-gather for large ones, fp32 or bf16 on the wire), launched on a
    dedicated comm stream with the 1/W average fused into the kernel.  Every bucket starts on a 16-byte
    boundary (parameters are padded to 4 elements) so buckets can be handed to the kernel as they are.

The fused NetResDeep engine (``parallel/ddp.py``) implements the same semantics inside its graph-captured step;
this wrapper is the path for arbitrary models and for CPU/gloo testing.
"""
from __future__ import annotations

import os
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn as nn


def _zero_flat(t: torch.Tensor) -> None:
    """Zero a flat (contiguous) gradient buffer: on a GPU one runtime fill on the current stream (no ATen kernel in
    the training step), else torch's zero_."""
    if t.is_cuda:
        from ..ops import _native as N
        N.check(N.lib().dca_ops_zero(N.ptr(t), t.numel() * t.element_size(), N.stream(t.device)), "zero")
    else:
        t.zero_()


def _dist_on(group=None) -> bool:
    return dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1


class FlatBucketDDP(nn.Module):
    def __init__(self, module: nn.Module, bucket_cap_mb: float = 4.0, first_bucket_mb: Optional[float] = 1.0,
                 broadcast_buffers: bool = True, process_group=None, device_ids=None, output_device=None,
                 comm: str = "auto", wire: str = "fp32", algo: str = "auto", loopback: bool = False):
        """``comm``: "auto" (xGMI for CUDA models when every rank is on this node, else the process group),
        "xgmi", or "process_group".  ``wire`` ("fp32" | "bf16") and ``algo`` ("auto" | "oneshot" | "twoshot")
        apply to the xGMI path.  ``loopback`` (one rank, CUDA): every bucket still goes through the xGMI
        communicator on the comm stream -- the rank is its own only peer -- so the per-bucket kernel's cost beside
        the backward is measurable on one device (``bench/resnet50.py --loopback``)."""
        super().__init__()
        if comm not in ("auto", "xgmi", "process_group"):
            raise ValueError("comm must be 'auto', 'xgmi' or 'process_group'")
        self.module = module
        self.process_group = process_group
        self.world_size = dist.get_world_size(process_group) if _dist_on(process_group) else 1
        self.broadcast_buffers = broadcast_buffers
        params = [p for _, p in module.named_parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        dev, dtype = params[0].device, params[0].dtype
        if any(p.device != dev or p.dtype != dtype for p in params):
            raise ValueError("FlatBucketDDP needs all parameters on one device with one dtype")
        order = list(reversed(params))  # approximately gradient-ready order
        total = sum((p.numel() + 3) // 4 * 4 for p in order)  # every parameter starts 16-byte aligned
        self.flat = torch.zeros(total, dtype=dtype, device=dev)
        self.flat_grad = torch.zeros(total, dtype=dtype, device=dev)
        self._views = {}
        off = 0
        with torch.no_grad():
            for p in order:
                n = p.numel()
                self.flat[off:off + n].copy_(p.detach().reshape(-1))
                p.data = self.flat[off:off + n].view_as(p)
                g = self.flat_grad[off:off + n].view_as(p)
                p.grad = g
                self._views[p] = (off, n, g)
                off += (n + 3) // 4 * 4
        # bucket plan: contiguous slices of the flat buffer
        esz = self.flat.element_size()
        cap = max(1, int(bucket_cap_mb * 2 ** 20 / esz))
        first_cap = max(1, int(first_bucket_mb * 2 ** 20 / esz)) if first_bucket_mb else cap
        self.buckets: List[tuple] = []  # (start, end, n_params)
        start, count, limit = 0, 0, first_cap
        cursor = 0
        for p in order:
            n = (p.numel() + 3) // 4 * 4
            if count and cursor + n - start > limit:
                self.buckets.append((start, cursor, count))
                start, count, limit = cursor, 0, cap
            cursor += n
            count += 1
        self.buckets.append((start, cursor, count))
        self._bucket_of = {}
        for bi, (s, e, _) in enumerate(self.buckets):
            for p in order:
                o = self._views[p][0]
                if s <= o < e:
                    self._bucket_of[p] = bi
        self._pending = [0] * len(self.buckets)
        self._ready = set()
        self._fused_opt = None  # FlatSGD(overlap=True): each bucket is updated as soon as it is reduced
        self._works: list = []
        self._callback_queued = False
        self.bucket_fire_order: List[int] = []  # for tests: order in which buckets were launched
        self._sync_next_forward = True
        self.timing = False  # True: record the comm-stream span of every step (comm_time(); metrics)
        self._comm_events: list = []
        self._flat_buffers = self._rehome_buffers(dev)
        self._sync_module_states()  # CC3
        self.comm, self.xgmi, self._comm_stream = "process_group" if self.world_size > 1 else "none", None, None
        self._wire, self._algo = wire, algo
        if loopback:
            if self.world_size != 1 or dev.type != "cuda" or dtype != torch.float32:
                raise ValueError("loopback: one rank, fp32 parameters on a GPU")
            from .xgmi import XgmiComm
            self.xgmi = XgmiComm.create(max(e - s for s, e, _ in self.buckets), group=process_group, device=dev,
                                        wire=wire)
            if self.xgmi is None:
                raise RuntimeError("xGMI loopback communicator unavailable")
            self.comm = "xgmi-loopback"
            self._comm_stream = torch.cuda.Stream(dev)
        elif self.world_size > 1 and dev.type == "cuda" and dtype == torch.float32 and comm != "process_group":
            local = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world_size)))
            if comm == "xgmi" or (local == self.world_size and self.world_size <= 8):
                from .xgmi import XgmiComm
                self.xgmi = XgmiComm.create(max(e - s for s, e, _ in self.buckets), group=process_group,
                                            device=dev, wire=wire)
                if self.xgmi is not None:
                    self.comm = "xgmi"
                    self._comm_stream = torch.cuda.Stream(dev)
        for p in order:
            p.register_post_accumulate_grad_hook(self._make_hook(p))
            # direct-write protocol (ops/functional.py grad_sink): a kernel that produces a parameter's whole
            # gradient for the step accumulates it into the flat view and reports readiness itself
            p._dca_grad_sink = (self._views[p][2], self._make_ready(p))

    # ---- collectives ------------------------------------------------------------------------------------------
    def _sync_module_states(self) -> None:
        if self.world_size == 1:
            return
        with torch.no_grad():
            dist.broadcast(self.flat, 0, group=self.process_group)
        self._broadcast_buffers_now()

    def _rehome_buffers(self, dev) -> list:
        """Module buffers (BN running mean / var, num_batches_tracked) become views of ONE flat tensor per dtype,
        like the parameters: CC4 is then one in-place broadcast per dtype -- no concatenation before it and no
        per-buffer copy after it (torch DDP coalesces into a temporary and copies back).  A buffer shared by
        several modules (NetResDeep's one ResBlock applied 10x) is re-homed once and stays shared.  Buffers on
        another device than the parameters keep their own storage (broadcast as they are)."""
        seen, groups = {}, {}
        for mod in self.module.modules():
            for name, b in mod._buffers.items():
                if b is None:
                    continue
                key = id(b)
                if key not in seen:
                    seen[key] = (b, [])
                    if b.device == dev:
                        groups.setdefault(b.dtype, []).append(key)
                seen[key][1].append((mod, name))
        flats = []
        with torch.no_grad():
            for dtype, keys in groups.items():
                total = sum(seen[k][0].numel() for k in keys)
                flat = torch.empty(total, dtype=dtype, device=dev)
                o = 0
                for k in keys:
                    b, users = seen[k]
                    n = b.numel()
                    v = flat[o:o + n].view_as(b)
                    v.copy_(b)
                    for mod, name in users:
                        mod._buffers[name] = v
                    o += n
                flats.append(flat)
        self._loose_buffers = [seen[k][0] for k in seen if seen[k][0].device != dev]
        return flats

    def _broadcast_buffers_now(self) -> None:
        if self.world_size == 1:
            return
        with torch.no_grad():
            for flat in self._flat_buffers:  # one in-place broadcast per dtype (the buffers are views of it)
                dist.broadcast(flat, 0, group=self.process_group)
            for b in self._loose_buffers:
                dist.broadcast(b, 0, group=self.process_group)

    def _make_hook(self, p):
        ready = self._make_ready(p)

        def hook(param):
            off, n, view = self._views[p]
            if param.grad is None or param.grad.data_ptr() != view.data_ptr():
                # optimizer.zero_grad(set_to_none=True) dropped the view; fold the fresh grad back in
                if param.grad is not None:
                    view.copy_(param.grad)
                param.grad = view
            ready()
        return hook

    def _make_ready(self, p):
        def ready():
            if self.world_size == 1 and self._fused_opt is None and self.xgmi is None:
                return
            # idempotent per step: a kernel-written (sink) gradient reports readiness itself, and autograd may
            # still run the parameter's AccumulateGrad with an undefined gradient, firing the hook as well
            if p in self._ready:
                return
            self._ready.add(p)
            if not self._callback_queued:
                torch.autograd.Variable._execution_engine.queue_callback(self._finish_backward)
                self._callback_queued = True
            bi = self._bucket_of[p]
            self._pending[bi] -= 1
            if self._pending[bi] == 0:
                self._launch(bi)
        return ready

    def _launch(self, bi: int) -> None:
        s, e, _ = self.buckets[bi]
        seg = self.flat_grad[s:e]
        if self.timing and seg.is_cuda and (self.world_size > 1 or self.xgmi is not None) and not self.bucket_fire_order:
            ev = torch.cuda.Event(enable_timing=True)  # first bucket of the step: comm span starts
            cs = self._side_stream()
            cs.wait_stream(torch.cuda.current_stream(seg.device))
            ev.record(cs)
            self._comm_events.append([ev, None])
        if self.world_size == 1 and self.xgmi is None:  # nothing to reduce: only the fused update (side stream on a GPU)
            if seg.is_cuda:
                cs = self._side_stream()
                cs.wait_stream(torch.cuda.current_stream(seg.device))
                with torch.cuda.stream(cs):
                    self._fused_opt._update_slice(s, e)
            else:
                self._fused_opt._update_slice(s, e)
        elif self.xgmi is not None:  # own xGMI all-reduce on the comm stream, average fused, no host sync
            cs = self._comm_stream
            cs.wait_stream(torch.cuda.current_stream(seg.device))
            self.xgmi.all_reduce_(seg, average=True, algo=self._algo, wire=self._wire, stream=cs)
            if self._fused_opt is not None:  # the bucket's SGD update right behind its all-reduce
                with torch.cuda.stream(cs):
                    self._fused_opt._update_slice(s, e)
        else:
            seg.div_(self.world_size)  # average: pre-divide, then sum
            work = dist.all_reduce(seg, group=self.process_group, async_op=True)
            if self._fused_opt is not None:
                if seg.is_cuda:  # ordered behind the collective on a side stream, overlapping the backward
                    with torch.cuda.stream(self._side_stream()):
                        work.wait()  # RCCL: a stream-level wait on the side stream, the host does not block
                        self._fused_opt._update_slice(s, e)
                    work = None
                else:
                    self._works.append((work, s, e))
                    work = None
            if work is not None:
                self._works.append((work, None, None))
        self.bucket_fire_order.append(bi)

    def _side_stream(self):
        if self._comm_stream is None:
            self._comm_stream = torch.cuda.Stream(self.flat.device)
        return self._comm_stream

    def _finish_backward(self) -> None:
        # parameters that received no gradient this step: reduce their (zero) slices too, in bucket order
        for bi, left in enumerate(self._pending):
            if left:
                self._launch(bi)
        for w, s, e in self._works:
            w.wait()
            if s is not None:  # CPU: the fused update of a bucket after its (gloo) all-reduce
                self._fused_opt._update_slice(s, e)
        if self._comm_stream is not None:
            if self._comm_events and self._comm_events[-1][1] is None:
                ev = torch.cuda.Event(enable_timing=True)
                ev.record(self._comm_stream)
                self._comm_events[-1][1] = ev
            torch.cuda.current_stream(self.flat_grad.device).wait_stream(self._comm_stream)
        self._works = []
        self._callback_queued = False
        self._reset_pending()

    def _reset_pending(self) -> None:
        self._pending = [b[2] for b in self.buckets]
        self._ready = set()

    # ---- module API -------------------------------------------------------------------------------------------
    def forward(self, *args, **kwargs):
        # CC4 with torch DDP's exact rule (nn/parallel/distributed.py require_forward_param_sync): a forward
        # broadcasts rank 0's buffers unless the PREVIOUS forward ran without autograd, so in an eval loop under
        # no_grad only the first batch runs a collective (a rank evaluating alone must use .module)
        if self.world_size > 1 and self.broadcast_buffers and self._sync_next_forward:
            self._broadcast_buffers_now()
        self._reset_pending()
        self.bucket_fire_order = []
        out = self.module(*args, **kwargs)
        self._sync_next_forward = torch.is_grad_enabled()
        return out

    def zero_grad(self, set_to_none: bool = False) -> None:  # grads stay views of the flat buffer
        _zero_flat(self.flat_grad)

    def comm_time(self, reset: bool = True) -> tuple:
        """(microseconds, steps) the gradient collectives spanned on the comm stream -- first bucket launched to
        backward finished -- over the timed steps since the last reset (``timing=True``; synchronises)."""
        tot, n = 0.0, 0
        for a, b in self._comm_events:
            if b is not None:
                b.synchronize()
                tot += a.elapsed_time(b) * 1e3
                n += 1
        if reset:
            self._comm_events = []
        return tot, n

    def check_comm(self) -> None:
        """Raise if the xGMI all-reduce recorded a peer timeout (synchronous; call at log points)."""
        if self.xgmi is not None:
            self.xgmi.check()

    def close(self) -> None:
        """Release the xGMI communicator (collective: every rank must call it)."""
        if self.xgmi is not None:
            self.xgmi.close()
            self.xgmi = None


class FlatSGD(torch.optim.Optimizer):
    """``optim.SGD`` over the flat buffer in one or two fused ops.

    Default = reference ``main.py:27`` (lr only).  ``momentum`` / ``weight_decay`` follow torch.optim.SGD's
    formulas (buf = m * buf + (g + wd * p); p -= lr * buf), e.g. the ppe_main_ddp.py setting SGD(1e-3, 0.9).

    ``overlap=True`` (BASELINE config 5, "fused SGD + all-reduce overlap"): every gradient bucket is updated as
    soon as it is complete -- right behind its all-reduce on the comm stream (HIP SGD kernel), or on a side
    stream with one rank -- so the update overlaps the rest of the backward; ``step()`` then has nothing left
    to do.  The momentum buffer starts at zero, so its first update equals the gradient (torch's semantics)."""

    def __init__(self, ddp: FlatBucketDDP, lr: float = 1e-2, momentum: float = 0.0, weight_decay: float = 0.0,
                 overlap: bool = False):
        super().__init__(list(ddp.module.parameters()), dict(lr=lr, momentum=momentum, weight_decay=weight_decay))
        self.ddp = ddp
        self._buf = None
        self.overlap = overlap
        if overlap:
            if ddp._fused_opt is not None:
                raise ValueError("FlatBucketDDP already has a fused optimizer")
            if momentum:
                self._buf = torch.zeros_like(ddp.flat)
            ddp._fused_opt = self

    @torch.no_grad()
    def _update_slice(self, s: int, e: int) -> None:
        g = self.param_groups[0]
        p, grad = self.ddp.flat[s:e], self.ddp.flat_grad[s:e]
        buf = self._buf[s:e] if self._buf is not None else None
        if p.is_cuda:
            from ..ops.functional import sgd_step_
            sgd_step_(p, grad, g["lr"], g["momentum"], g["weight_decay"], buf=buf, first=None)
            return
        d = grad.add(p, alpha=g["weight_decay"]) if g["weight_decay"] else grad
        if buf is not None:
            buf.mul_(g["momentum"]).add_(d)
            d = buf
        p.add_(d, alpha=-g["lr"])

    @torch.no_grad()
    def step(self, closure=None):
        loss = closure() if closure is not None else None
        if self.overlap:  # already applied bucket by bucket during the backward
            return loss
        g = self.param_groups[0]
        if self.ddp.flat.is_cuda:  # one HIP kernel over the flat buffer (ops/functional.py sgd_step_)
            from ..ops.functional import sgd_step_
            if g["momentum"] and self._buf is None:
                self._buf = torch.empty_like(self.ddp.flat)
                self._first = torch.ones(1, dtype=torch.int32, device=self.ddp.flat.device)
            sgd_step_(self.ddp.flat, self.ddp.flat_grad, g["lr"], g["momentum"], g["weight_decay"], buf=self._buf,
                      first=getattr(self, "_first", None))
            return loss
        grad = self.ddp.flat_grad
        if g["weight_decay"]:
            grad = grad.add(self.ddp.flat, alpha=g["weight_decay"])
        if g["momentum"]:
            if self._buf is None:
                self._buf = grad.clone()
            else:
                self._buf.mul_(g["momentum"]).add_(grad)
            grad = self._buf
        self.ddp.flat.add_(grad, alpha=-g["lr"])
        return loss

    def zero_grad(self, set_to_none: bool = True) -> None:
        _zero_flat(self.ddp.flat_grad)
