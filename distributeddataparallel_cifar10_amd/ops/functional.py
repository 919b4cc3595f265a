"""Autograd functions over the ops-layer HIP kernels (csrc/ops_*.hip).

Activations are channels-last bf16 tensors ``[N, H, W, C]`` (contiguous); parameters stay fp32 in the module
layout of torch (``Conv2d.weight [Cout, Cin, KH, KW]``, ``Linear.weight [out, in]``) so ``state_dict`` is the
reference's.  GEMMs run on MFMA (bf16, or fp8 e4m3 for the forward when ``fp8=True``) with fp32 accumulation;
BatchNorm statistics are fp32.

Reference ops: conv2d K1/K4/K19/K22, BatchNorm2d + ReLU + residual K5-K7/K17/K18/K20,
max_pool2d K3/K16, linear K9/K10/K13/K15, cross-entropy K11/K12, SGD K24.
"""
from __future__ import annotations

import math
import os
from typing import Optional

import torch

from . import _native as N


_BWD_TRACE = None  # diagnostics: a list to record the order of the fused conv-BN backward calls
WGRAD_NARROW_HALF = True  # _wgrad_splits' halved target for the narrow forms (False: the round-6 rule, for A/Bs)
# the row-ring weight gradient of the 64-channel 3x3 convs (csrc/ops_wgrad.hip k_wgrad3x3_rows) is on unless either
# of its native knobs turns it off; it sets that form's split count (_wgrad_splits)
WGRAD_ROWS = os.environ.get("DCA_OPS_WGRAD_ROWS", "1") != "0" and os.environ.get("DCA_OPS_CONV_ROWS", "1") != "0"


def _dev_check(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("ops kernels need GPU tensors")


# ------------------------------------------------------------------------------------------------------------
# GEMM
# ------------------------------------------------------------------------------------------------------------
def gemm(a: torch.Tensor, b: torch.Tensor, *, ta: bool = False, tb: bool = False, bias: Optional[torch.Tensor] = None,
         relu: bool = False, out_dtype=torch.float32, alpha: float = 1.0, out: Optional[torch.Tensor] = None,
         beta: float = 0.0, splits: int = 0, alpha_dev: Optional[torch.Tensor] = None, conv: int = 0,
         geom=None, col_stats: Optional[torch.Tensor] = None, stats_shift: Optional[torch.Tensor] = None,
         mnk=None, amax_a: Optional[torch.Tensor] = None, amax_b: Optional[torch.Tensor] = None,
         wperm=None, orow=None, beta_src: Optional[torch.Tensor] = None,
         beta_mask: Optional[torch.Tensor] = None) -> torch.Tensor:
    """C[M,N] = alpha * A(m,k) B(n,k) (+bias) (+beta*out) (ReLU).

    A is [M,K] (ta=False) or [K,M] (ta=True); B is [N,K] (tb=False) or [K,N] (tb=True).  bf16 operands, or
    fp8 e4m3 stored as uint8 (both, K-contiguous).  splits=0 chooses split-K automatically.
    conv=1 / conv=2: A / B is an NHWC input gathered as im2col on the fly (``geom`` = conv geometry, ``mnk`` =
    the GEMM shape).  col_stats [ceil(M/128), N, 2] fp32 receives per-tile BN partial sums of the output.
    amax_a / amax_b: fp8 per-tensor amax bits (int32 [1]) of the operands, folded into alpha on the device.
    wperm = (C, Cpad, T): weight-gradient output written straight into torch's [M, C, KH, KW] fp32 layout
    (``out``), GEMM column n = tap * Cpad + c; padded channels dropped.
    orow = (S, ph, pw, H, W, Ho, Wo): row m = pixel (n, i, j) of an Ho x Wo grid goes to row
    (n H + S i + ph) W + S j + pw of ``out`` ([N H W, N_gemm]): a strided conv's sub-pixel input gradient."""
    _dev_check(a, b, bias, out)
    fp8 = a.dtype == torch.uint8
    if fp8 != (b.dtype == torch.uint8) or (not fp8 and (a.dtype != torch.bfloat16 or b.dtype != torch.bfloat16)):
        raise TypeError("gemm operands: both bf16 or both fp8 (uint8)")
    if conv:
        M, Nn, K = mnk
    else:
        if a.dim() != 2 or b.dim() != 2 or a.stride(1) != 1 or b.stride(1) != 1:
            raise ValueError("gemm operands must be 2-D with unit inner stride")
        M, K = (a.shape[1], a.shape[0]) if ta else (a.shape[0], a.shape[1])
        Nn, Kb = (b.shape[1], b.shape[0]) if tb else (b.shape[0], b.shape[1])
        if K != Kb:
            raise ValueError(f"gemm: K mismatch {K} vs {Kb}")
    if wperm is not None:
        if out is None or out.dtype != torch.float32 or not out.is_contiguous() \
                or out.numel() != M * wperm[0] * wperm[2]:
            raise ValueError("gemm: weight-layout output must be contiguous fp32 [M, C, KH, KW]")
    elif orow is not None:
        if out is None or out.dim() != 2 or out.shape[1] != Nn or not out.is_contiguous() \
                or out.shape[0] != M // (orow[5] * orow[6]) * orow[3] * orow[4]:
            raise ValueError("gemm: remapped output must be contiguous [N*H*W, N_gemm]")
    else:
        if out is None:
            out = torch.empty(M, Nn, dtype=out_dtype, device=a.device)
        if out.dtype not in (torch.float32, torch.bfloat16) or out.shape != (M, Nn) or out.stride(1) != 1:
            raise ValueError("gemm: bad output tensor")
    if bias is not None and (bias.dtype != torch.float32 or bias.numel() != Nn):
        raise ValueError("gemm: bias must be fp32 [N]")
    tiles = math.ceil(M / 128) * math.ceil(Nn / 128)
    if col_stats is not None or orow is not None:
        splits = 1
    if splits <= 0:
        splits = 1
        kt = 128 if fp8 else 64
        if tiles < 256 and K >= 4 * kt:
            splits = max(1, min(K // (2 * kt), 512 // tiles, 64))
    ws = torch.empty(splits * M * Nn, dtype=torch.float32, device=a.device) \
        if splits > 1 or wperm is not None else None
    args = N.GemmArgs(A=a.data_ptr(), B=b.data_ptr(), C=out.data_ptr(), bias=bias.data_ptr() if bias is not None else None,
                      ws=ws.data_ptr() if ws is not None else None, M=M, N=Nn, K=K,
                      lda=a.stride(0) if a.dim() == 2 else 0, ldb=b.stride(0) if b.dim() == 2 else 0,
                      ldc=Nn if wperm is not None else out.stride(0), alpha=float(alpha), beta=float(beta), ta=int(ta),
                      tb=int(tb), fp8=int(fp8), relu=int(relu), out_bf16=int(out.dtype == torch.bfloat16),
                      splits=splits, k_per_split=0,
                      alpha_dev=alpha_dev.data_ptr() if alpha_dev is not None else None, conv=int(conv),
                      col_stats=col_stats.data_ptr() if col_stats is not None else None,
                      stats_shift=stats_shift.data_ptr() if stats_shift is not None else None,
                      amax_a=amax_a.data_ptr() if amax_a is not None else None,
                      amax_b=amax_b.data_ptr() if amax_b is not None else None)
    if wperm is not None:
        args.wperm_C, args.wperm_Cpad, args.wperm_T = (int(v) for v in wperm)
    if orow is not None:
        (args.orow_S, args.orow_ph, args.orow_pw, args.orow_H, args.orow_W, args.orow_Ho,
         args.orow_Wo) = (int(v) for v in orow)
    if conv:
        for f in ("N", "H", "W", "C", "KH", "KW", "Ho", "Wo"):
            setattr(args, "c" + f, getattr(geom, f))
        args.cS, args.cP = geom.stride, geom.pad
    if beta_mask is not None:  # C = A B + beta * (beta_src * mask bits): beta_src has C's [M, ldc] layout
        if beta_src is None or beta_src.dtype != torch.bfloat16 or not beta_src.is_contiguous() \
                or beta_src.numel() != M * Nn or beta_mask.numel() * 8 != M * Nn or out.stride(0) != Nn:
            raise ValueError("gemm: masked accumulation source must be a contiguous bf16 [M, N] tensor + M*N/8 bytes")
        args.beta_src, args.beta_mask = beta_src.data_ptr(), beta_mask.data_ptr()
    N.check(N.lib().dca_ops_gemm(args, N.stream(a.device)), "gemm")
    return out


def quantize_fp8(x: torch.Tensor):
    """Per-tensor fp8 e4m3 quantisation on the device: (q uint8 same shape, amax bits int32 [1]).
    q = sat(x * 448 / amax); dequantise with amax / 448."""
    _dev_check(x)
    x = x.contiguous()
    q = torch.empty(x.shape, dtype=torch.uint8, device=x.device)
    amax = torch.empty(1, dtype=torch.int32, device=x.device)
    if x.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError("quantize_fp8: fp32 or bf16 input")
    N.check(N.lib().dca_ops_quant_fp8(N.ptr(x), int(x.dtype == torch.float32), x.numel(), N.ptr(q), N.ptr(amax),
                                      N.stream(x.device)), "quant_fp8")
    return q, amax


def fp8_alpha(amax_a: torch.Tensor, amax_b: torch.Tensor, extra: float = 1.0) -> torch.Tensor:
    out = torch.empty(1, dtype=torch.float32, device=amax_a.device)
    N.check(N.lib().dca_ops_fp8_alpha(N.ptr(amax_a), N.ptr(amax_b), float(extra), N.ptr(out), N.stream(amax_a.device)),
            "fp8_alpha")
    return out


def amax_value(amax_bits: torch.Tensor) -> torch.Tensor:
    return amax_bits.view(torch.float32)


def _wgrad_splits(M: int, Nn: int, K: int, implicit: bool = False, row_w: int = 0) -> int:
    """Split-K factor for a weight-gradient GEMM (K = pixels: long, M x N small): enough workgroups to fill the
    chip twice over (2 resident per CU x 256 CUs), >= 4 K-tiles per split, fp32 slab <= 64 MiB.  Half that target
    for the plain 64-wide forms (k_wgrad 64 x 128 / 128 x 64 / 64 x 64 tiles: 802816 x {64, 256} x {64, 256}
    53 -> 43, 116 -> 99, 115 -> 101 us) and the 128-channel implicit 3x3 ones (k_wgrad_pp: 144 -> 134, 120 ->
    116 us), where the partial slabs and their reduce cost more than the extra workgroups hide
    (profiles/wgrad_split_sweep_r8c.log; the 64-channel implicit 3x3 wants the full target: 148 vs 200 us).
    The 64-channel implicit 3x3 on input rows of row_w <= 64 pixels runs k_wgrad3x3_rows, one split slab per
    workgroup: 512 splits = two workgroups per CU (its launcher takes min(splits, 2 x CUs, rows)); the 128-channel
    one on rows <= 32 pixels two workgroups per slab, one per CU: 128 splits; the s2d stem's (k_wgrad_s2d_rows)
    three per CU: 768 (150 -> 143 us over 512; 128 / 96 / 64 and 512 / 384 / 256 for the 3x3 forms measured slower:
    profiles/wgrad_rows_splits_r9q.log).  row_w: input row width of a KH > 1 implicit conv, else 0."""
    if implicit and M == 64 and Nn == 576 and 0 < row_w <= 64 and WGRAD_ROWS:
        return max(1, min(512, K // 256))
    if implicit and M == 128 and Nn == 1152 and 0 < row_w <= 32 and WGRAD_ROWS:  # layer 2: 2 workgroups per split
        return max(1, min(128, K // 256))
    if implicit and M == 64 and Nn == 256 and 0 < row_w <= 128 and WGRAD_ROWS:  # s2d stem: 3 workgroups per CU
        return max(1, min(768, K // 256))
    tiles = math.ceil(M / 128) * math.ceil(Nn / 128)
    narrow = (min(M, Nn) <= 64) if not implicit else (min(M, Nn) == 128)
    s = math.ceil((512 if narrow and WGRAD_NARROW_HALF else 1024) / tiles)
    s = min(s, K // 256, max(1, (64 << 20) // (4 * M * Nn)))
    return max(1, s)


def dy_prep(dy: torch.Tensor, y: Optional[torch.Tensor] = None, want_bf16: bool = True, want_db: bool = True,
            db_into: Optional[torch.Tensor] = None):
    """Backward preamble of a GEMM layer in one launch: dy [.., N] (fp32 / bf16) masked by ReLU(y > 0) when y is
    given -> (dy as a bf16 GEMM operand or None, db = column sums fp32 [N] or None).  Replaces the cast, the mask
    multiply and the bias-gradient reduction (three ATen kernels).  db_into: accumulate the column sums into this
    fp32 view instead (a flat DDP gradient sink)."""
    _dev_check(dy, y)
    dy = dy.contiguous()
    n = dy.shape[-1]
    r = dy.numel() // n
    dyb = torch.empty(dy.shape, dtype=torch.bfloat16, device=dy.device) if want_bf16 else None
    if db_into is not None:
        db = db_into
    else:  # (without want_db: still one launch, the column sums go to a scratch vector)
        db = torch.empty(n, dtype=torch.float32, device=dy.device)
    ncb = (n + 63) // 64  # 64-column blocks
    nchunk = max(1, min((1024 + ncb - 1) // ncb, (r + 15) // 16))  # ~1024 workgroups, >= 16 rows each
    part = torch.empty(nchunk * n, dtype=torch.float32, device=dy.device)
    if y is not None:
        y = y.contiguous()
    N.check(N.lib().dca_ops_dy_prep(N.ptr(dy), int(dy.dtype == torch.bfloat16), N.ptr(y),
                                    int(y is not None and y.dtype == torch.bfloat16), N.ptr(dyb), N.ptr(part),
                                    N.ptr(db), N.ptr(_ticket(dy.device, ncb)), r, n, nchunk, int(db_into is not None),
                                    N.stream(dy.device)), "dy_prep")
    return dyb, (db if want_db and db_into is None else None)


def zeros_bf16(*shape, device) -> torch.Tensor:
    """A zeroed bf16 tensor by one runtime fill (no ATen fill kernel in the step)."""
    t = torch.empty(*shape, dtype=torch.bfloat16, device=device)
    N.check(N.lib().dca_ops_zero(N.ptr(t), t.numel() * 2, N.stream(device)), "zero")
    return t


def gather_cols(src: torch.Tensor, idx: torch.Tensor, out: torch.Tensor, accumulate: bool) -> None:
    """out[r, j] (+)= src[r, idx[j]] for 2-D fp32 src [rows, S] / out [rows, L] (contiguous), one launch."""
    rows, S = src.shape
    L = idx.numel()
    N.check(N.lib().dca_ops_gather_cols(N.ptr(src), S, N.ptr(idx), L, N.ptr(out), rows, int(accumulate),
                                        N.stream(src.device)), "gather_cols")


def add_one_i64(ptrs: torch.Tensor, n: int) -> None:
    """``*ptrs[i] += 1`` for the n int64 counters whose addresses ``ptrs`` (a device int64 tensor) holds: every
    BatchNorm's num_batches_tracked in one launch."""
    N.check(N.lib().dca_ops_add_i64(N.ptr(ptrs), int(n), N.stream(ptrs.device)), "add_i64")


def cast_bf16(x: torch.Tensor) -> torch.Tensor:
    """fp32 -> bf16 (RNE) on the ops kernels (a weight operand outside the WeightPack)."""
    _dev_check(x)
    x = x.contiguous()
    y = torch.empty(x.shape, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib().dca_ops_cast_bf16(N.ptr(x), N.ptr(y), x.numel(), N.stream(x.device)), "cast_bf16")
    return y


# ------------------------------------------------------------------------------------------------------------
# Linear (x [B, in] bf16, w [out, in] fp32 master) -> fp32 or bf16
# ------------------------------------------------------------------------------------------------------------
class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, relu, out_dtype, fp8, sinks):
        xb = x.contiguous() if x.dtype == torch.bfloat16 else cast_bf16(x.float())
        wb = cast_bf16(w.detach())
        if fp8:
            qx, ax = quantize_fp8(xb)
            qw, aw = quantize_fp8(wb)
            y = gemm(qx, qw, bias=b, relu=relu, out_dtype=out_dtype, amax_a=ax, amax_b=aw)
        else:
            y = gemm(xb, wb, bias=b, relu=relu, out_dtype=out_dtype)
        ctx.save_for_backward(xb, wb, y if relu else None)
        ctx.relu, ctx.has_b, ctx.sinks = relu, b is not None, sinks
        return y

    @staticmethod
    def backward(ctx, dy):
        xb, wb, y = ctx.saved_tensors
        sw, sb = ctx.sinks if ctx.sinks is not None else (None, None)
        want_db = ctx.has_b and (ctx.needs_input_grad[2] or sb is not None)
        # ReLU mask, bf16 operand and the bias gradient (into its flat DDP view when sunk) in one launch
        dyb, db = dy_prep(dy, y if ctx.relu else None, want_db=want_db, db_into=sb[0] if sb is not None else None)
        dx = dw = None
        if ctx.needs_input_grad[0]:
            dx = gemm(dyb, wb, tb=True, out_dtype=torch.bfloat16)  # dX = dY . W
        if ctx.needs_input_grad[1] or sw is not None:
            M, Nn, K = wb.shape[0], wb.shape[1], xb.shape[0]
            splits = _wgrad_splits(M, Nn, K)
            if sw is not None:  # dW = dY^T . X accumulated by the GEMM's reduce pass into the flat gradient view
                gemm(dyb, xb, ta=True, tb=True, splits=splits, out=sw[0], beta=1.0)
            else:
                dw = gemm(dyb, xb, ta=True, tb=True, splits=splits)  # dW = dY^T . X (fp32)
        for sink in (sw, sb):
            if sink is not None:
                sink[1]()
        ctx.sinks = None
        return dx, dw, db, None, None, None, None


def linear(x, w, b=None, relu=False, out_dtype=torch.float32, fp8=False):
    """x [B, in] -> [B, out].  Under FlatBucketDDP (grad sinks on w and b) the weight and bias gradients are written
    straight into the flat gradient buffer by the backward's kernels (no autograd accumulate kernels)."""
    sinks = None
    if torch.is_grad_enabled() and b is not None:
        sw, sb = grad_sink(w), grad_sink(b)
        if sw is not None and sb is not None and sw[0].is_contiguous():
            sinks = (sw, sb)
    return _Linear.apply(x, w, b, relu, out_dtype, fp8, sinks)


# ------------------------------------------------------------------------------------------------------------
# Conv2d, NHWC: im2col (or the input itself for 1x1/stride 1) + MFMA GEMM; bias and ReLU fused in the epilogue
# ------------------------------------------------------------------------------------------------------------
def _geom(x, w, stride, pad):
    n, h, wd, c = x.shape
    co, ci, kh, kw = w.shape
    if ci != c and not (ci < c and c % 8 == 0 and ci <= 8):  # a 3-channel stem may arrive zero-padded to 8
        raise ValueError(f"conv: input has {c} channels, weight expects {ci}")
    ho, wo = (h + 2 * pad - kh) // stride + 1, (wd + 2 * pad - kw) // stride + 1
    k = kh * kw * c
    kp = (k + 7) // 8 * 8
    return N.ConvGeom(N=n, H=h, W=wd, C=c, KH=kh, KW=kw, stride=stride, pad=pad, Ho=ho, Wo=wo, K=k, Kp=kp)


def _weight_matrix(w: torch.Tensor, kp: int) -> torch.Tensor:
    """[Cout, Cin, KH, KW] fp32 -> [Cout, Kp] bf16 with column k = (kh*KW + kw)*Cin + ci (zero padded)."""
    co = w.shape[0]
    m = w.permute(0, 2, 3, 1).reshape(co, -1)
    if m.shape[1] != kp:
        m = torch.nn.functional.pad(m, (0, kp - m.shape[1]))
    return m.to(torch.bfloat16).contiguous()


def _implicit_ok(g) -> bool:
    return g.C % 8 == 0


class WeightPack:
    """The bf16 (and fp8) GEMM operands of every convolution of a model, rebuilt from the fp32 master weights
    by ONE kernel launch per step (``pack()``; csrc/ops_nn.hip k_pack_weights / k_pack_fp8) instead of a
    permute / pad / cast chain per layer and per use.

    Per conv: ``fwd`` [Cout, KH*KW*Cin_pad] (forward, strided input gradient), ``dgrad`` [Cin, KH*KW*Cout]
    (flipped; stride-1 input gradient: an implicit conv for KxK, a plain NT GEMM with W^T for 1x1) and, for ``fp8`` layers, ``q8`` + ``amax``.
    Cin_pad = 8 for a stem with fewer than 8 channels (its input is zero-padded to 8 channels, so the stem runs
    as an implicit GEMM instead of through an im2col buffer)."""

    BLOCKS_PER_LAYER = 256

    def __init__(self, convs, fp8_convs=(), s2d_convs=()):
        self.convs = list(convs)
        fp8_ids = {id(c) for c in fp8_convs}
        s2d_ids = {id(c) for c in s2d_convs}
        self.entries = {}
        n_fp8 = sum(1 for c in self.convs if id(c) in fp8_ids)
        dev = self.convs[0].weight.device
        self.amax = torch.zeros(max(1, n_fp8), dtype=torch.int32, device=dev)
        j = 0
        for c in self.convs:
            co, ci, kh, kw = c.weight.shape
            ci_pad = ci if ci % 8 == 0 else (ci + 7) // 8 * 8
            kp = kh * kw * ci_pad
            e = dict(ci_pad=ci_pad, kp=kp, fwd=torch.empty(co, kp, dtype=torch.bfloat16, device=dev), dgrad=None,
                     q8=None, amax=None)
            if ci_pad == ci and co % 8 == 0 and ((c.stride[0] == 1 and (kh > 1 or c.padding[0] == 0))
                                                 or (c.stride[0] == 2 and kh == 1 and c.padding[0] == 0)):
                e["dgrad"] = torch.empty(ci, kh * kw * co, dtype=torch.bfloat16, device=dev)
            e["classes"] = None
            if c.stride == (2, 2) and kh > 1 and kh == kw and ci_pad == ci and co % 8 == 0:
                e["classes"] = self._parity_classes(c, dev)
            if id(c) in fp8_ids:
                e["q8"] = torch.empty(co, kp, dtype=torch.uint8, device=dev)
                e["amax"] = self.amax[j:j + 1]
                j += 1
            e["s2d"] = None
            if id(c) in s2d_ids:  # space-to-depth stem: [Co, 4 * 4 * 16] gathered from w (no dgrad: network input)
                idx_f, idx_b = stem_s2d_index(c)
                e.update(ci_pad=S2D_C, kp=S2D_TAPS * S2D_TAPS * S2D_C, dgrad=None, classes=None, q8=None, amax=None,
                         fwd=torch.empty(co, S2D_TAPS * S2D_TAPS * S2D_C, dtype=torch.bfloat16, device=dev),
                         s2d=dict(shape=(co, S2D_C, S2D_TAPS, S2D_TAPS), fwd_idx=idx_f, back_idx=idx_b))
            self.entries[id(c)] = e
        self.n_fp8 = n_fp8
        self._key = None
        self._descs = None
        self._gkey = None
        self._n_gather = 0

    @staticmethod
    def _parity_classes(c, dev):
        """Sub-pixel decomposition of a stride-2 conv's input gradient: input pixels of parity (ph, pw) receive
        dY only through the taps kh with (ph + pad - kh) even, from dY row i + (ph + pad - kh) / 2.  Each class
        is a stride-1 implicit conv over dY (taps ordered by that offset, pad = -min offset) with the matrix
        [Cin][(a_h KWc + a_w) Cout + co] = w[co][ci][kh_a][kw_a]; returns [(ph, pw, KHc, KWc, pad, out, idx)]."""
        import numpy as np
        co, ci, k, _ = c.weight.shape
        p = c.padding[0]

        def taps(par):
            t = sorted(((par + p - kk) // 2, kk) for kk in range(k) if (par + p - kk) % 2 == 0)
            return [kk for _, kk in t], -t[0][0]

        out = []
        for ph in (0, 1):
            for pw in (0, 1):
                (kh_l, pad_h), (kw_l, pad_w) = taps(ph), taps(pw)
                if pad_h != pad_w:
                    return None
                o_, c_, ah, aw = np.meshgrid(np.arange(co), np.arange(ci), np.arange(len(kh_l)), np.arange(len(kw_l)),
                                             indexing="ij")
                src = ((o_ * ci + c_) * k + np.asarray(kh_l)[ah]) * k + np.asarray(kw_l)[aw]  # w[co][ci][kh][kw]
                col = (ah * len(kw_l) + aw) * co + o_
                idx = np.empty((ci, len(kh_l) * len(kw_l) * co), dtype=np.int32)
                idx[c_, col] = src
                out.append((ph, pw, len(kh_l), len(kw_l), pad_h,
                            torch.empty(idx.shape, dtype=torch.bfloat16, device=dev),
                            torch.from_numpy(idx.reshape(-1)).to(dev)))
        return out

    def get(self, conv):
        return self.entries.get(id(conv))

    def pack(self) -> None:
        key = tuple(c.weight.data_ptr() for c in self.convs)
        packed = [c for c in self.convs if self.entries[id(c)]["s2d"] is None]
        if key != self._key and packed:  # parameters re-pointed (e.g. into a flat DDP buffer): rebuild descriptors
            arr = (N.PackDesc * len(packed))()
            for i, c in enumerate(packed):
                e = self.entries[id(c)]
                co, ci, kh, kw = c.weight.shape
                if not c.weight.is_contiguous():
                    raise ValueError("WeightPack: conv weights must be contiguous")
                if max(co * e["kp"], ci * kh * kw * co) + 4096 * 256 >= 2 ** 31:
                    raise ValueError("WeightPack: layer too large for the 32-bit pack kernel indices")
                arr[i] = N.PackDesc(w=c.weight.data_ptr(), fwd=e["fwd"].data_ptr(),
                                    dgrad=e["dgrad"].data_ptr() if e["dgrad"] is not None else None,
                                    q8=e["q8"].data_ptr() if e["q8"] is not None else None,
                                    amax=e["amax"].data_ptr() if e["amax"] is not None else None,
                                    co=co, ci=ci, ci_pad=e["ci_pad"], kh=kh, kw=kw, kp=e["kp"])
            host = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8)
            self._descs = host.to(self.amax.device)
            self._key = key
        if packed:
            N.check(N.lib().dca_ops_pack_weights(N.ptr(self._descs), len(packed), self.BLOCKS_PER_LAYER,
                                                 N.ptr(self.amax), self.n_fp8, N.stream(self.amax.device)),
                    "pack_weights")
        if key != self._gkey:
            # (weight, index table, output): strided-dgrad parity classes and space-to-depth stem matrices
            gl = [(c, cl[6], cl[5]) for c in self.convs for cl in (self.entries[id(c)]["classes"] or [])]
            gl += [(c, e["s2d"]["fwd_idx"], e["fwd"]) for c in self.convs
                   for e in [self.entries[id(c)]] if e["s2d"] is not None]
            self._n_gather = len(gl)
            if gl:
                arr = (N.GatherDesc * len(gl))()
                for i, (c, idx, out) in enumerate(gl):
                    arr[i] = N.GatherDesc(w=c.weight.data_ptr(), idx=idx.data_ptr(), out=out.data_ptr(),
                                          n=out.numel())
                self._gdescs = torch.frombuffer(bytearray(bytes(arr)), dtype=torch.uint8).to(self.amax.device)
            self._gkey = key
        if self._n_gather:
            N.check(N.lib().dca_ops_pack_gather(N.ptr(self._gdescs), self._n_gather, 64, N.stream(self.amax.device)),
                    "pack_gather")


def nchw_to_nhwc8(x: torch.Tensor) -> torch.Tensor:
    """Network input NCHW fp32 (C <= 8) -> NHWC bf16 with the channels zero-padded to 8, in one kernel (the
    implicit-GEMM stem's operand).  The input needs no gradient."""
    _dev_check(x)
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] > 8:
        raise ValueError("nchw_to_nhwc8: NCHW fp32 with at most 8 channels")
    x = x.contiguous()
    n, c, h, w = x.shape
    y = torch.empty(n, h, w, 8, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib().dca_ops_nchw_to_nhwc8(N.ptr(x), N.ptr(y), n, c, h * w, N.stream(x.device)), "nchw_to_nhwc8")
    return y


def stem_s2d_ok(conv: torch.nn.Conv2d) -> bool:
    """A 7x7 / 2 convolution with padding 3 over <= 4 input channels (the ResNet stem): it runs as a 4x4 stride-1
    conv over the space-to-depth input (``nchw_to_s2d16``), K = 4 x 4 taps x 16 channels = 256 instead of
    7 x 7 x 8 = 392."""
    return (conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3) and conv.in_channels <= 4
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None)


S2D_TAPS, S2D_C, S2D_PAD = 4, 16, 4  # 4x4 taps of 16 channels; input shifted by padding + 1 = 4 (even)


def stem_s2d_index(conv: torch.nn.Conv2d):
    """Index tables between the stem weight w [Co, C, 7, 7] and its space-to-depth form w' [Co, 16, 4, 4] (torch
    layout of the 4x4 conv; GEMM column (i * 4 + j) * 16 + ch of the forward matrix): channel ch = (2 ph + pw) C + c
    of tap (i, j) holds w[:, c, 2i + ph - 1, 2j + pw - 1] (zero where that lies outside 0..6).
    Returns (fwd [Co * 256] int32: source element of every forward-matrix entry, -1 for zero;
             back [C * 49] int64: column of w'.view(Co, 256) that holds (c, kh, kw))."""
    import numpy as np
    co, ci = conv.weight.shape[:2]
    fwd = np.full((co, S2D_TAPS, S2D_TAPS, S2D_C), -1, dtype=np.int32)
    back = np.zeros((ci, 7, 7), dtype=np.int64)
    for i in range(S2D_TAPS):
        for j in range(S2D_TAPS):
            for ph in (0, 1):
                for pw in (0, 1):
                    kh, kw = 2 * i + ph - 1, 2 * j + pw - 1
                    if not (0 <= kh < 7 and 0 <= kw < 7):
                        continue
                    for c in range(ci):
                        ch = (2 * ph + pw) * ci + c
                        fwd[:, i, j, ch] = (np.arange(co) * ci + c) * 49 + kh * 7 + kw
                        back[c, kh, kw] = ch * S2D_TAPS * S2D_TAPS + i * S2D_TAPS + j
    dev = conv.weight.device
    return torch.from_numpy(fwd.reshape(-1)).to(dev), torch.from_numpy(back.reshape(-1)).to(dev)


def nchw_to_s2d16(x: torch.Tensor) -> torch.Tensor:
    """Network input NCHW fp32 (C <= 4) -> the space-to-depth NHWC bf16 operand of the 7x7/2/3 stem
    ([N, Ho + 3, Wo + 3, 16], one kernel).  The input needs no gradient."""
    _dev_check(x)
    if x.dtype != torch.float32 or x.dim() != 4 or x.shape[1] > 4:
        raise ValueError("nchw_to_s2d16: NCHW fp32 with at most 4 channels")
    x = x.contiguous()
    n, c, h, w = x.shape
    ho, wo = (h + 6 - 7) // 2 + 1, (w + 6 - 7) // 2 + 1
    hs, ws = ho + S2D_TAPS - 1, wo + S2D_TAPS - 1
    y = torch.empty(n, hs, ws, S2D_C, dtype=torch.bfloat16, device=x.device)
    N.check(N.lib().dca_ops_nchw_to_s2d16(N.ptr(x), N.ptr(y), n, c, h, w, hs, ws, S2D_PAD, N.stream(x.device)),
            "nchw_to_s2d16")
    return y


def _s2d_args(w, stride, pad, packed):
    """(geometry weight, stride, pad) of a conv: its own, or for a space-to-depth stem entry the 4x4 / 1 / 0 conv
    over the s2d input (a meta tensor carries the shape)."""
    if packed is not None and packed.get("s2d") is not None:
        return torch.empty(packed["s2d"]["shape"], device="meta"), 1, 0
    return w, stride, pad


def grad_sink(p: torch.Tensor):
    """(flat gradient view, ready callback) that FlatBucketDDP attaches to its parameters, or None.  A kernel
    that owns a parameter's whole gradient for the step writes (accumulates) it straight into the view and
    signals readiness, so no gradient tensor is materialised and no accumulate kernel runs."""
    return getattr(p, "_dca_grad_sink", None)


class GradJoin:
    """A tensor consumed by ``n`` ops-layer functions (a ResNet block input: conv1 and the identity path / the
    downsample conv) whose input gradients must be summed.  Instead of autograd's separate add kernel, the
    first producer writes the gradient buffer and returns None; later producers accumulate into it inside their
    own kernel (GEMM beta = 1, col2im accumulate); the last one returns the sum."""

    def __init__(self, n: int = 2, defer_ok: bool = False):
        self.buf = None
        self.left = n
        # defer_ok: the first producer may register (dout, ReLU bit mask) instead of writing dout * mask; the
        # next producer (a 1x1 conv's dgrad GEMM) then takes it as its masked accumulation source
        self.defer_ok = defer_ok
        self.masked = None

    def defer_masked(self, src, mask):
        """First producer: the gradient is src * mask (bits); nothing written.  Returns None (not the last)."""
        if self.buf is not None or self.masked is not None or not self.defer_ok:
            raise RuntimeError("GradJoin: a masked contribution must come first, once, and be allowed")
        self.masked = (src, mask)
        self.left -= 1
        if self.left <= 0:
            raise RuntimeError("GradJoin: the masked contribution needs a later producer")
        return None

    def take_masked(self):
        m, self.masked = self.masked, None
        return m

    def contribute(self, t):
        """Register a producer's result (the buffer itself when it accumulated); returns what that producer
        hands to autograd."""
        if self.buf is None:
            self.buf = t
        elif t is not self.buf:
            raise RuntimeError("GradJoin: a later producer must accumulate into the shared buffer")
        self.left -= 1
        if self.left < 0:
            raise RuntimeError("GradJoin: more producers than declared")
        return self.buf if self.left == 0 else None


# The downsample branch's BN applied on the fly by bn3's apply pass (ResidualLink.lazy); False: the branch writes
# its BN output and bn3 reads it (A/B comparisons: DCA_OPS_RES_BN=0)
RES_BN_ON_THE_FLY = os.environ.get("DCA_OPS_RES_BN", "1") != "0"


class ResidualLink:
    """ReLU(bn3 + r) of a downsample bottleneck -> the downsample branch that produced r.  bn3's backward leaves
    (dout, its forward ReLU bit mask) here and returns no gradient for r, so dL/dr = dout * mask is never written;
    the downsample BN's backward (called by autograd with no gradient: its forward disables grad materialisation)
    reads dout and the mask instead (k_bn_bwd_* in BWD_MASK mode).  Forward: the branch's BN only finalises its
    statistics and hands (its conv output, statistics, gamma, beta) over ``lazy``; bn3's apply pass normalises the
    residual on the fly, so the branch's BN output is never written."""

    def __init__(self):
        self.dout = self.mask = None
        # forward: (conv output data_ptr, stats, gamma, beta) of the branch's BN, applied by bn3 on the fly
        self.lazy = None


class Fp8Delayed:
    """Delayed-scaling fp8 state of ONE activation tensor feeding ONE fp8 GEMM (Transformer-Engine style).

    The producer (a fused BN apply) writes the fp8 copy with scale 448 / amax_prev -- the previous step's amax --
    and records this step's amax; the consumer GEMM dequantises with amax_prev, then promotes the new amax for the
    next step.  All on the device: no host sync, no extra pass over the activation.  Before the first amax is
    known the consumer quantises the tensor itself (``quantize_fp8``) and seeds the state."""

    def __init__(self):
        self.amax_prev = None   # fp32 [1]
        self.amax_out = None    # int32 [1] (float bits) written by the producer
        self.q = None           # fp8 copy emitted for the current step
        self.src_ptr = 0        # data_ptr of the bf16 tensor it is a copy of

    @property
    def ready(self) -> bool:
        return self.amax_prev is not None


def _fp8_operand(cols, state: Optional["Fp8Delayed"]):
    """(q, amax bits) of the activation operand: the producer's delayed-scaled copy when there is one."""
    if state is not None and state.q is not None and state.src_ptr == cols.data_ptr() \
            and state.q.numel() == cols.numel():
        q, bits = state.q.view(cols.shape), state.amax_prev.view(torch.int32)
        state.q = None
        return q, bits, True
    q, bits = quantize_fp8(cols)
    if state is not None and not state.ready:
        state.amax_prev = bits.view(torch.float32).clone()
        state.amax_out = torch.zeros(1, dtype=torch.int32, device=cols.device)
    return q, bits, False


def _conv_fwd(x, w, b, stride, pad, relu, fp8, col_stats=None, shift=None, fp8_state=None, packed=None):
    """Forward GEMM of a conv; returns (y [N,Ho,Wo,Cout] bf16, state for _conv_bwd).  ``packed``: this conv's
    WeightPack entry (pre-built bf16 / fp8 operands) or None (operands built here from the fp32 weight)."""
    x = x.contiguous()
    g = _geom(x, w, stride, pad)
    co = w.shape[0]
    M = g.N * g.Ho * g.Wo
    direct = w.shape[2] == 1 and w.shape[3] == 1 and stride == 1 and pad == 0
    st = dict(geom=g, wshape=tuple(w.shape), x=x, cols=None, packed=packed)
    if packed is not None and packed["kp"] != g.K:
        raise ValueError("conv: packed weight does not match the input channels")
    use_fp8 = fp8 and g.Kp % 16 == 0 and (packed is None or packed["q8"] is not None)
    if use_fp8 and not direct and g.C % 16 == 0 and packed is not None:
        # fp8 implicit conv: the NHWC input's fp8 copy (emitted by its producer) gathered on the fly
        qx, ax, delayed = _fp8_operand(x, fp8_state)
        y = gemm(qx, packed["q8"], conv=1, geom=g, mnk=(M, co, g.K), bias=b, relu=relu, out_dtype=torch.bfloat16,
                 amax_a=ax, amax_b=packed["amax"], col_stats=col_stats, stats_shift=shift)
        if delayed:
            fp8_state.amax_prev.copy_(fp8_state.amax_out.view(torch.float32))
        st["wm"] = packed["fwd"]
        return y.view(g.N, g.Ho, g.Wo, co), st
    if direct or use_fp8 or not _implicit_ok(g):
        if direct:
            cols = x.view(M, g.K)
        else:
            cols = torch.empty(M, g.Kp, dtype=torch.bfloat16, device=x.device)
            N.check(N.lib().dca_ops_im2col(N.ptr(x), N.ptr(cols), g, N.stream(x.device)), "im2col")
        st["cols"] = cols
        wm = packed["fwd"] if packed is not None and g.Kp == g.K else _weight_matrix(w, g.Kp)
        if use_fp8:
            qc, ac, delayed = _fp8_operand(cols, fp8_state)
            if packed is not None:
                qw, aw = packed["q8"], packed["amax"]
            else:
                qw, aw = quantize_fp8(wm)
            y = gemm(qc, qw, bias=b, relu=relu, out_dtype=torch.bfloat16, amax_a=ac, amax_b=aw,
                     col_stats=col_stats, stats_shift=shift)
            if delayed:  # this step's amax (recorded by the producer) scales the next step
                fp8_state.amax_prev.copy_(fp8_state.amax_out.view(torch.float32))
        else:
            y = gemm(cols, wm, bias=b, relu=relu, out_dtype=torch.bfloat16, col_stats=col_stats, stats_shift=shift)
    else:  # implicit GEMM: the im2col matrix is never materialised
        wm = packed["fwd"] if packed is not None else _weight_matrix(w, g.K)
        y = gemm(x, wm, conv=1, geom=g, mnk=(M, co, g.K), bias=b, relu=relu, out_dtype=torch.bfloat16,
                 col_stats=col_stats, stats_shift=shift)
    st["wm"] = wm
    return y.view(g.N, g.Ho, g.Wo, co), st


def _unmask(src: torch.Tensor, mask: torch.Tensor) -> torch.Tensor:
    """src * mask bits (bit j of byte e / 8 = element e) as a new bf16 tensor: the masked-copy kernel through a
    zero-K-free path (a 1x1 GEMM would need weights), used only when a deferred join meets a non-1x1 consumer."""
    bits = (mask.view(-1, 1) >> torch.arange(8, device=mask.device, dtype=torch.uint8)) & 1
    return (src.reshape(-1) * bits.view(-1).to(src.dtype)).view_as(src).contiguous()


def _conv_bwd(dy, st, need_x: bool, need_w: bool, sink=None, x_join: Optional[GradJoin] = None):
    """(dx, dw) of a conv from dY [N,Ho,Wo,Cout] (any dtype) and the forward state.  The weight gradient is
    written by the GEMM's reduce pass directly in torch's [Cout, Cin, KH, KW] layout -- into ``sink`` (a flat
    gradient view, accumulated; dw returned as None) when given.  ``x_join``: the input is shared with another
    consumer; its gradient is accumulated into (or seeds) the join's buffer (dx None until the last producer)."""
    g, (co, ci, kh, kw) = st["geom"], st["wshape"]
    packed = st.get("packed")
    M = g.N * g.Ho * g.Wo
    dyb = dy.to(torch.bfloat16).contiguous().view(M, co)
    dx = dw = None
    cols = st["cols"]
    if need_x:
        acc = x_join.buf if x_join is not None else None  # accumulate into the other consumer's gradient
        masked = x_join.take_masked() if x_join is not None and x_join.masked is not None else None
        if masked is not None and not (cols is not None and cols.data_ptr() == st["x"].data_ptr()):
            acc = _unmask(*masked)  # (only the 1x1 dgrad below takes the masked source in its epilogue)
            masked = None
        beta = 1.0 if acc is not None or masked is not None else 0.0
        dst2 = acc.view(g.N * g.H * g.W, g.C) if acc is not None else None
        if cols is not None and cols.data_ptr() == st["x"].data_ptr():  # 1x1 / stride 1: dX = dY . W
            msrc, mbits = (masked[0].view(M, g.C), masked[1]) if masked is not None else (None, None)
            if packed is not None and packed["dgrad"] is not None:  # W^T [Cin, Cout] from the pack: plain NT
                dx = gemm(dyb, packed["dgrad"], out_dtype=torch.bfloat16, out=dst2, beta=beta,
                          beta_src=msrc, beta_mask=mbits)
            else:
                dx = gemm(dyb, st["wm"], tb=True, out_dtype=torch.bfloat16, out=dst2, beta=beta,
                          beta_src=msrc, beta_mask=mbits)
            dx = dx.view(g.N, g.H, g.W, g.C)
        elif g.stride == 1 and co % 8 == 0 and kh == kw and g.pad <= kh - 1 and g.C == ci:
            # stride 1: dX = conv(dY, W flipped, ci<->co, pad KH-1-pad), implicit GEMM (no col2im)
            gd = N.ConvGeom(N=g.N, H=g.Ho, W=g.Wo, C=co, KH=kh, KW=kw, stride=1, pad=kh - 1 - g.pad, Ho=g.H, Wo=g.W,
                            K=kh * kw * co, Kp=kh * kw * co)
            if packed is not None and packed["dgrad"] is not None:
                wd = packed["dgrad"]
            else:
                wd = st.get("w_master").flip(2, 3).permute(1, 2, 3, 0).reshape(ci, -1).to(torch.bfloat16).contiguous()
            dx = gemm(dyb.view(g.N, g.Ho, g.Wo, co), wd, conv=1, geom=gd, mnk=(g.N * g.H * g.W, ci, gd.K),
                      out_dtype=torch.bfloat16, out=dst2, beta=beta).view(g.N, g.H, g.W, g.C)
        elif (packed is not None and g.stride == 2 and g.H % 2 == 0 and g.W % 2 == 0 and g.C == ci
              and (packed.get("classes") or (kh == 1 and g.pad == 0 and packed["dgrad"] is not None))):
            # sub-pixel decomposition: each parity class of input pixels is a stride-1 implicit conv over dY whose
            # GEMM epilogue writes straight into its rows of dX (no dY.W^T column matrix, no col2im)
            classes = packed["classes"] or [(0, 0, 1, 1, 0, packed["dgrad"], None)]
            if acc is None:
                dx = torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=dy.device) if len(classes) == 4 \
                    else zeros_bf16(g.N, g.H, g.W, g.C, device=dy.device)
            else:
                dx = acc
            dy4 = dyb.view(g.N, g.Ho, g.Wo, co)
            for ph, pw, nkh, nkw, pad_c, wc, _ in classes:
                ho_c, wo_c = (g.H - ph + 1) // 2, (g.W - pw + 1) // 2
                gc = N.ConvGeom(N=g.N, H=g.Ho, W=g.Wo, C=co, KH=nkh, KW=nkw, stride=1, pad=pad_c, Ho=ho_c, Wo=wo_c,
                                K=nkh * nkw * co, Kp=nkh * nkw * co)
                rows = g.N * ho_c * wo_c
                gemm(dy4, wc, conv=1, geom=gc, mnk=(rows, ci, gc.K), out=dx.view(-1, ci), beta=beta,
                     orow=(2, ph, pw, g.H, g.W, ho_c, wo_c))
        else:
            wm = st["wm"]
            dcols = gemm(dyb, wm, tb=True, out_dtype=torch.bfloat16)  # [M, Kp] = dY . Wm
            kp = wm.shape[1]
            gc = N.ConvGeom(N=g.N, H=g.H, W=g.W, C=g.C, KH=g.KH, KW=g.KW, stride=g.stride, pad=g.pad, Ho=g.Ho,
                            Wo=g.Wo, K=g.K, Kp=kp)
            dx = acc if acc is not None else torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=dy.device)
            N.check(N.lib().dca_ops_col2im(N.ptr(dcols), N.ptr(dx), gc, int(acc is not None), N.stream(dy.device)),
                    "col2im")
        if x_join is not None:
            dx = x_join.contribute(dx if acc is None else acc)  # (a masked source: dx is the fresh sum)
    if need_w:
        dst = sink if sink is not None else torch.empty(co, ci, kh, kw, dtype=torch.float32, device=dy.device)
        beta = 1.0 if sink is not None else 0.0
        perm = (ci, g.C, kh * kw)
        if cols is not None:
            kp = cols.shape[1]
            gemm(dyb, cols, ta=True, tb=True, splits=_wgrad_splits(co, kp, M), out=dst, beta=beta, wperm=perm)
        else:  # implicit: B(n = tap*C + c, k = pixel) gathered from x
            gemm(dyb, st["x"], ta=True, conv=2, geom=g, mnk=(co, g.K, M),
                 splits=_wgrad_splits(co, g.K, M, True, row_w=g.W if g.KH > 1 else 0), out=dst, beta=beta,
                 wperm=perm)
        dw = None if sink is not None else dst
    return dx, dw


class _Conv2d(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, stride, pad, relu, fp8):
        y, st = _conv_fwd(x, w, b, stride, pad, relu, fp8)
        st["w_master"] = w.detach()
        ctx.st = st
        ctx.save_for_backward(y if relu else None)
        ctx.relu, ctx.has_b = relu, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        db = None
        if ctx.relu or (ctx.has_b and ctx.needs_input_grad[2]):  # ReLU mask + bias gradient: one launch
            dy, db = dy_prep(dy, y if ctx.relu else None, want_db=ctx.has_b and ctx.needs_input_grad[2])
        dx, dw = _conv_bwd(dy, ctx.st, ctx.needs_input_grad[0], ctx.needs_input_grad[1])
        ctx.st = None
        return dx, dw, db, None, None, None, None


class _ConvBNAct(torch.autograd.Function):
    """conv (no bias) -> BatchNorm (train) -> ReLU / residual, with the BN statistics computed in the conv
    GEMM's epilogue (no separate statistics pass over the conv output)."""

    @staticmethod
    def forward(ctx, x, w, r, gamma, beta, running_mean, running_var, stride, pad, eps, momentum, relu, res_mode, fp8,
                fp8_state, emit, packed, sinks, x_join, r_join, res_in, pool):
        ctx.res_in = res_in
        if res_in is not None:  # the consumer may hand this output's gradient over res_in instead of autograd
            ctx.set_materialize_grads(False)
        co = w.shape[0]
        wg, stride, pad = _s2d_args(w, stride, pad, packed)
        g = _geom(x, wg, stride, pad)
        M = g.N * g.Ho * g.Wo
        nparts = (M + 127) // 128
        part = torch.empty(nparts, co, 2, dtype=torch.float32, device=x.device)
        y, st = _conv_fwd(x, wg, None, stride, pad, False, fp8, col_stats=part, shift=running_mean,
                          fp8_state=fp8_state, packed=packed)
        st["w_master"] = w.detach()
        stats = torch.empty(co, 2, dtype=torch.float32, device=x.device)
        ctx.st = st
        ctx.wshape = tuple(w.shape)
        ctx.sinks = sinks
        ctx.joins = (x_join, r_join)
        ctx.relu, ctx.res_mode = relu, res_mode
        ctx.pool = None
        if pool:  # ReLU(bn(y)) -> 3x3/2/1 max pool in one pass: the activation itself is never written
            pg = _pool_geom(y, 3, 2, 1)
            out = torch.empty(pg.N, pg.Ho, pg.Wo, co, dtype=torch.bfloat16, device=x.device)
            arg = torch.empty(pg.N, pg.Ho, pg.Wo, co, dtype=torch.uint8, device=x.device)
            N.check(N.lib().dca_ops_bn_pool_fwd_parts(N.ptr(y), N.ptr(part), nparts, N.ptr(stats), N.ptr(gamma),
                                                      N.ptr(beta), N.ptr(running_mean), N.ptr(running_var),
                                                      float(eps), float(momentum), N.ptr(out), N.ptr(arg), pg,
                                                      N.ptr(_ticket(x.device, (co + 63) // 64)), N.stream(x.device)),
                    "bn_pool_fwd_parts")
            ctx.pool = pg
            ctx.save_for_backward(y, None, gamma, beta, stats, arg)
            return out
        r = r.contiguous() if r is not None else None
        # the downsample branch of a bottleneck (its output is only bn3's residual, over a ResidualLink): statistics
        # only, the conv output y is returned and bn3's apply normalises it on the fly (k_bn_apply BnRes)
        lazy = (RES_BN_ON_THE_FLY and isinstance(res_in, ResidualLink) and not relu and res_mode == 0 and r is None
                and emit is None)
        # bn3 of that block: its residual r is such a raw conv output
        rl = (r_join.lazy if isinstance(r_join, ResidualLink) and r_join.lazy is not None and r is not None and
              r_join.lazy[0] == r.data_ptr() and res_mode == 2 else None)
        out = None if lazy else torch.empty_like(y)
        q = None
        if emit is not None and emit.ready:  # fp8 copy of the output for the next (fp8) GEMM, delayed scaling
            q = torch.empty(y.shape, dtype=torch.uint8, device=x.device)
        # ReLU(bn + r): the forward stores the ReLU mask as bits, so the backward reads M*C/8 bytes instead of r
        mask = torch.empty(M * co // 8, dtype=torch.uint8, device=x.device) if relu and res_mode == 2 else None
        N.check(N.lib().dca_ops_bn_fwd_parts(N.ptr(y), N.ptr(r), N.ptr(out), N.ptr(part), nparts, N.ptr(stats),
                                             N.ptr(gamma), N.ptr(beta), N.ptr(running_mean), N.ptr(running_var), M, co,
                                             float(eps), float(momentum), int(relu), int(res_mode), N.ptr(q),
                                             N.ptr(emit.amax_prev) if q is not None else None,
                                             N.ptr(emit.amax_out) if q is not None else None, N.ptr(mask),
                                             *((N.ptr(t) for t in rl[1:]) if rl is not None else (None,) * 3),
                                             N.ptr(_ticket(x.device, (co + 63) // 64)), N.stream(x.device)),
                "bn_fwd_parts")
        if q is not None:
            emit.q, emit.src_ptr = q, out.data_ptr()
        if rl is not None:
            r_join.lazy = None
        ctx.save_for_backward(y, r if mask is None else None, gamma, beta, stats, mask)
        if lazy:
            res_in.lazy = (y.data_ptr(), stats, gamma, beta)
            return y
        return out

    @staticmethod
    def backward(ctx, dout):
        y, r, gamma, beta, stats, mask = ctx.saved_tensors
        in_mask = None
        if dout is None:  # (res_in: grad materialisation is off) the consumer's bn3 left dout and its mask
            rl = ctx.res_in
            if rl is None or rl.dout is None:
                ctx.st = ctx.sinks = ctx.joins = ctx.res_in = None
                return (None,) * 22
            dout, in_mask, rl.dout, rl.mask = rl.dout, rl.mask, None, None
        if _BWD_TRACE is not None:
            _BWD_TRACE.append((tuple(y.shape), in_mask is not None))
        sw, sg, sb = ctx.sinks if ctx.sinks is not None else (None, None, None)
        x_join, r_join = ctx.joins
        res_link = isinstance(r_join, ResidualLink) and mask is not None and ctx.res_mode == 2
        defer = (not res_link and r_join is not None and mask is not None and r_join.defer_ok
                 and ctx.res_mode == 2)
        dout = dout.to(torch.bfloat16).contiguous()
        if ctx.pool is not None:  # dout is the pooled gradient; `mask` holds the pool's argmax bytes
            dy_conv, dgamma, dbeta = _bn_pool_backward(dout, mask, y, gamma, beta, stats, ctx.pool,
                                                       dgamma_out=sg[0] if sg else None,
                                                       dbeta_out=sb[0] if sb else None)
            dr = None
        else:
            dy_conv, dr, dgamma, dbeta = _bn_backward(dout, y, r, gamma, beta, stats, ctx.relu, ctx.res_mode,
                                                      dgamma_out=sg[0] if sg else None,
                                                      dbeta_out=sb[0] if sb else None,
                                                      mask=mask if in_mask is None else in_mask,
                                                      want_dr=not (defer or res_link))
        if sg:
            sg[1]()
            sb[1]()
        if res_link:  # dL/dr = dout * mask goes to the downsample branch through the link: never written
            r_join.dout, r_join.mask, dr = dout, mask, None
        elif defer:  # the identity gradient dout * mask is taken by conv1's dgrad epilogue: never written
            dr = r_join.defer_masked(dout, mask)
        elif r_join is not None and dr is not None:  # the identity gradient seeds the block input's shared buffer
            dr = r_join.contribute(dr)
        s2d = (ctx.st.get("packed") or {}).get("s2d")
        dx, dw = _conv_bwd(dy_conv, ctx.st, ctx.needs_input_grad[0], ctx.needs_input_grad[1] or sw is not None,
                           sink=sw[0] if sw and s2d is None else None,
                           x_join=x_join if ctx.needs_input_grad[0] else None)
        if s2d is not None and dw is not None:  # [Co, 16, 4, 4] of the 4x4 conv -> the stem's [Co, C, 7, 7]
            co = dw.shape[0]
            src = dw.reshape(co, -1).contiguous()
            if sw:  # one gather-accumulate launch straight into the flat gradient view
                gather_cols(src, s2d["back_idx"], sw[0].view(co, -1), accumulate=True)
                dw = None
            else:
                out = torch.empty(ctx.wshape, dtype=torch.float32, device=src.device)
                gather_cols(src, s2d["back_idx"], out.view(co, -1), accumulate=False)
                dw = out
        if sw:
            sw[1]()
        ctx.st = ctx.sinks = ctx.joins = ctx.res_in = None
        return (dx, dw, dr, dgamma, dbeta, None, None, None, None, None, None, None, None, None, None, None, None, None,
                None, None, None, None)


def conv_bn_act(x, conv: torch.nn.Conv2d, bn: torch.nn.BatchNorm2d, r=None, relu=True, fp8=False, res_mode=None,
                fp8_state: Optional[Fp8Delayed] = None, emit: Optional[Fp8Delayed] = None, packed=None,
                direct_grads: bool = False, x_join: Optional[GradJoin] = None, r_join: Optional[GradJoin] = None,
                res_in: Optional[ResidualLink] = None, pool: bool = False):
    """act(bn(conv(x))) for NHWC bf16 x, conv without bias (BN in eval mode: inference under no_grad, running
    statistics); with a residual r: res_mode 2 (default,
    ResNet: act(bn + r)) or 1 (NetResDeep: act(bn) + r).  fp8: forward GEMM in fp8 e4m3 (fp8_state: this conv's
    delayed-scaling input state); emit: also produce the fp8 copy of the output that the consumer of ``emit`` reads.
    packed: the conv's WeightPack entry.  direct_grads: the conv weight and BN affine parameters are used once
    per step, so their gradients may be written straight into FlatBucketDDP's flat buffer (``grad_sink``).
    x_join / r_join: the input x / the residual r is also consumed elsewhere (GradJoin): its gradient is summed
    inside the producing kernels instead of by an autograd add.  pool: follow with the 3x3 / stride 2 / pad 1 max
    pool (the ResNet stem) in the same pass when ``bn_pool_ok`` (training, ReLU, no residual; else a separate
    pool): returns the pooled tensor, and neither the activation nor its gradient is ever materialised.  (Measured and removed in round 5: the BN-backward
    statistics in the consumer's dgrad GEMM epilogue, 8,417 vs 8,755 img/s at ResNet-50 batch 256.)"""
    if res_mode is None:
        res_mode = 2 if r is not None else 0
    if conv.bias is not None:
        raise ValueError("conv_bn_act: conv without bias")
    _check_join(bn, relu, res_mode)
    if not bn.training:  # inference: running statistics, no autograd
        _check_inference(conv.weight)
        with torch.no_grad():
            wg, stride, pad = _s2d_args(conv.weight, conv.stride[0], conv.padding[0], packed)
            y, _ = _conv_fwd(x, wg, None, stride, pad, False, False, packed=packed)
            out = _bn_eval(y, r, bn, relu, res_mode)
            return max_pool2d(out, 3, 2, 1) if pool else out
    momentum = bn.momentum if bn.track_running_stats else 0.0
    if bn.track_running_stats and not getattr(bn, "_dca_counted", False):
        bn.num_batches_tracked.add_(1)  # (a model that batches these increments marks its BNs _dca_counted)
    sinks = None
    if direct_grads and torch.is_grad_enabled():
        sw, sg, sb = grad_sink(conv.weight), grad_sink(bn.weight), grad_sink(bn.bias)
        if sw is not None and sg is not None and sb is not None:
            sinks = (sw, sg, sb)
    fuse = pool and relu and r is None and res_mode == 0 and emit is None and BN_POOL_FUSED and \
        bn_pool_ok(x, conv, packed)
    out = _ConvBNAct.apply(x, conv.weight, r, bn.weight, bn.bias, bn.running_mean, bn.running_var, conv.stride[0],
                           conv.padding[0], bn.eps, momentum, relu, res_mode, fp8, fp8_state, emit, packed, sinks,
                           x_join if torch.is_grad_enabled() else None, r_join if torch.is_grad_enabled() else None,
                           res_in if torch.is_grad_enabled() else None, fuse)
    return max_pool2d(out, 3, 2, 1) if pool and not fuse else out


def conv2d(x, w, b=None, stride=1, pad=0, relu=False, fp8=False):
    """x: [N, H, W, Cin] bf16 (NHWC); w: [Cout, Cin, KH, KW] fp32 -> [N, Ho, Wo, Cout] bf16."""
    return _Conv2d.apply(x, w, b, stride, pad, relu, fp8)


# ------------------------------------------------------------------------------------------------------------
# BatchNorm (train) + ReLU + residual, NHWC bf16.  res_mode 0: act(bn(x)); 1: act(bn(x)) + r; 2: act(bn(x) + r)
# ------------------------------------------------------------------------------------------------------------
class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, r, gamma, beta, running_mean, running_var, eps, momentum, relu, res_mode):
        x = x.contiguous()
        C = x.shape[-1]
        M = x.numel() // C
        r = r.contiguous() if r is not None else None
        out = torch.empty_like(x)
        part = torch.empty((M + 255) // 256, C, 2, dtype=torch.float32, device=x.device)
        stats = torch.empty(C, 2, dtype=torch.float32, device=x.device)
        N.check(N.lib().dca_ops_bn_fwd(N.ptr(x), N.ptr(r), N.ptr(out), N.ptr(part), N.ptr(stats), N.ptr(gamma),
                                       N.ptr(beta), N.ptr(running_mean), N.ptr(running_var), M, C, float(eps),
                                       float(momentum), int(relu), int(res_mode), N.ptr(_ticket(x.device, (C + 63) // 64)),
                                       N.stream(x.device)), "bn_fwd")
        ctx.save_for_backward(x, r, gamma, beta, stats)
        ctx.relu, ctx.res_mode = relu, res_mode
        return out

    @staticmethod
    def backward(ctx, dy):
        x, r, gamma, beta, stats = ctx.saved_tensors
        dx, dr, dgamma, dbeta = _bn_backward(dy, x, r, gamma, beta, stats, ctx.relu, ctx.res_mode)
        return dx, dr, dgamma, dbeta, None, None, None, None, None, None


def _bn_backward(dy, x, r, gamma, beta, stats, relu, res_mode, dgamma_out=None, dbeta_out=None,
                 mask=None, want_dr: bool = True):
    """(dx, dr, dgamma, dbeta) of the fused BN + ReLU + residual.  dgamma_out / dbeta_out: flat gradient views
    to accumulate into (then dgamma / dbeta are returned as None).  mask: the forward's ReLU bit mask (res_mode 2;
    r is then not needed)."""
    dy = dy.to(torch.bfloat16).contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    part = torch.empty((M + 255) // 256, C, 2, dtype=torch.float32, device=x.device)
    sums = torch.empty(C, 2, dtype=torch.float32, device=x.device)
    direct = dgamma_out is not None and dbeta_out is not None
    dgamma = dgamma_out if direct else torch.empty(C, dtype=torch.float32, device=x.device)
    dbeta = dbeta_out if direct else torch.empty_like(dgamma)
    dx = torch.empty_like(x)
    # without dr (mask given): the residual's consumer reads dy and the mask itself (GradJoin.defer_masked)
    dr = torch.empty_like(x) if res_mode == 2 and (want_dr or mask is None) else None
    N.check(N.lib().dca_ops_bn_bwd(N.ptr(dy), N.ptr(x), N.ptr(r), N.ptr(stats), N.ptr(gamma), N.ptr(beta),
                                   N.ptr(part), N.ptr(sums), N.ptr(dgamma), N.ptr(dbeta), N.ptr(dx), N.ptr(dr),
                                   M, C, int(relu), int(res_mode), int(direct), N.ptr(mask),
                                   N.ptr(_ticket(x.device, (C + 63) // 64)), N.stream(x.device)),
            "bn_bwd")
    if res_mode == 1:
        dr = dy
    if direct:
        return dx, dr, None, None
    return dx, dr, dgamma, dbeta


# The ResNet stem's BN + ReLU + max pool in one pass (k_bn_pool_fwd / k_bn_pool_bwd_*); False: BN apply and the
# pool as two passes each way (A/B comparisons: DCA_OPS_STEM_POOL=0)
BN_POOL_FUSED = os.environ.get("DCA_OPS_STEM_POOL", "1") != "0"


def _pool_geom(x: torch.Tensor, k: int, s: int, p: int):
    n, h, w, c = x.shape
    return N.PoolGeom(N=n, H=h, W=w, C=c, K=k, S=s, P=p, Ho=(h + 2 * p - k) // s + 1, Wo=(w + 2 * p - k) // s + 1)


def bn_pool_ok(x: torch.Tensor, conv: torch.nn.Conv2d, packed=None) -> bool:
    """The conv's output can take the fused BN + ReLU + 3x3/2/1 max pool: even H and W (every input pixel in the
    2x2 block of one output pixel), C % 64 == 0, 32-bit element offsets."""
    if not x.is_cuda:
        return False
    wg, stride, pad = _s2d_args(conv.weight, conv.stride[0], conv.padding[0], packed)
    g = _geom(x, wg, stride, pad)
    co = conv.out_channels
    return (g.Ho % 2 == 0 and g.Wo % 2 == 0 and co % 64 == 0 and
            g.N * g.Ho * g.Wo * co + 8192 * 256 < 2 ** 31)


def _bn_pool_backward(dp, arg, y, gamma, beta, stats, pg, dgamma_out=None, dbeta_out=None):
    """(dy, dgamma, dbeta) of ReLU(BN(y)) -> max pool from the pooled gradient dp and the argmax bytes; dgamma_out /
    dbeta_out: flat gradient views accumulated into (then dgamma / dbeta are None)."""
    C = y.shape[-1]
    npo = pg.N * pg.Ho * pg.Wo
    part = torch.empty((npo + 63) // 64, C, 2, dtype=torch.float32, device=y.device)
    sums = torch.empty(C, 2, dtype=torch.float32, device=y.device)
    direct = dgamma_out is not None and dbeta_out is not None
    dgamma = dgamma_out if direct else torch.empty(C, dtype=torch.float32, device=y.device)
    dbeta = dbeta_out if direct else torch.empty_like(dgamma)
    dy = torch.empty_like(y)
    N.check(N.lib().dca_ops_bn_pool_bwd(N.ptr(dp), N.ptr(arg), N.ptr(y), N.ptr(stats), N.ptr(gamma), N.ptr(beta),
                                        N.ptr(part), N.ptr(sums), N.ptr(dgamma), N.ptr(dbeta), N.ptr(dy), int(direct),
                                        pg, N.ptr(_ticket(y.device, (C + 63) // 64)), N.stream(y.device)),
            "bn_pool_bwd")
    return dy, (None if direct else dgamma), (None if direct else dbeta)


def _check_inference(p: torch.Tensor) -> None:
    if torch.is_grad_enabled() and p.requires_grad:
        raise RuntimeError("ops layer: eval-mode BatchNorm is the inference path; run it under torch.no_grad() "
                           "(training-mode BN for gradients)")


def _bn_eval(x, r, bn: torch.nn.BatchNorm2d, relu, res_mode):
    """Eval-mode BatchNorm2d (normalised with the running statistics) + ReLU / residual over NHWC bf16 x, the
    same k_bn_apply pass as training with the statistics taken from the running buffers (torch BatchNorm2d eval
    semantics; reference model/resnet.py:28 in ``model.eval()``)."""
    if not bn.track_running_stats or bn.running_mean is None:
        raise NotImplementedError("ops eval BatchNorm needs running statistics")
    x = x.contiguous()
    C = x.shape[-1]
    M = x.numel() // C
    r = r.contiguous() if r is not None else None
    out = torch.empty_like(x)
    stats = torch.empty(C, 2, dtype=torch.float32, device=x.device)
    N.check(N.lib().dca_ops_bn_eval(N.ptr(x), N.ptr(r), N.ptr(out), N.ptr(stats), N.ptr(bn.weight), N.ptr(bn.bias),
                                    N.ptr(bn.running_mean), N.ptr(bn.running_var), M, C, float(bn.eps), int(relu),
                                    int(res_mode), N.stream(x.device)), "bn_eval")
    return out


def _check_join(bn, relu, res_mode):
    """Training: act(bn + r) (res_mode 2) exists only WITH the ReLU -- its backward kernels recover the residual
    gradient through the ReLU mask -- so the combination is refused here, before a forward whose backward would
    fail (eval-mode inference supports it)."""
    if res_mode == 2 and not relu and bn.training and torch.is_grad_enabled():
        raise ValueError("res_mode 2 (bn + r) without ReLU is not supported in training; use relu=True or res_mode 1")


def batch_norm_act(x, bn: torch.nn.BatchNorm2d, r=None, relu=True, res_mode=0):
    """BatchNorm2d `bn` over NHWC x.  Training mode: batch statistics, running stats updated in place,
    num_batches_tracked += 1.  Eval mode: running statistics (inference, under no_grad)."""
    if res_mode and r is None:
        raise ValueError("batch_norm_act: residual mode needs r")
    _check_join(bn, relu, res_mode)
    if not bn.training:  # inference: running statistics, no autograd
        _check_inference(bn.weight)
        with torch.no_grad():
            return _bn_eval(x, r if res_mode else None, bn, relu, res_mode)
    momentum = bn.momentum if bn.track_running_stats else 0.0
    if bn.track_running_stats:
        bn.num_batches_tracked.add_(1)
    return _BatchNormAct.apply(x, r if res_mode else None, bn.weight, bn.bias, bn.running_mean, bn.running_var,
                               bn.eps, momentum, relu, res_mode)


# ------------------------------------------------------------------------------------------------------------
# Pooling
# ------------------------------------------------------------------------------------------------------------
class _MaxPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, k, s, p):
        x = x.contiguous()
        n, h, w, c = x.shape
        ho, wo = (h + 2 * p - k) // s + 1, (w + 2 * p - k) // s + 1
        g = N.PoolGeom(N=n, H=h, W=w, C=c, K=k, S=s, P=p, Ho=ho, Wo=wo)
        y = torch.empty(n, ho, wo, c, dtype=torch.bfloat16, device=x.device)
        arg = torch.empty(n, ho, wo, c, dtype=torch.uint8, device=x.device)
        N.check(N.lib().dca_ops_maxpool_fwd(N.ptr(x), N.ptr(y), N.ptr(arg), g, N.stream(x.device)), "maxpool_fwd")
        ctx.save_for_backward(arg)
        ctx.geom = g
        return y

    @staticmethod
    def backward(ctx, dy):
        (arg,) = ctx.saved_tensors
        g = ctx.geom
        dy = dy.to(torch.bfloat16).contiguous()
        dx = torch.empty(g.N, g.H, g.W, g.C, dtype=torch.bfloat16, device=dy.device)
        N.check(N.lib().dca_ops_maxpool_bwd(N.ptr(dy), N.ptr(arg), N.ptr(dx), g, N.stream(dy.device)), "maxpool_bwd")
        return dx, None, None, None


def max_pool2d(x, k=2, s=None, p=0):
    return _MaxPool.apply(x, k, s or k, p)


class _AvgPool(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, out_bf16):
        if x.dtype != torch.bfloat16 or x.dim() != 4:
            raise ValueError("global_avg_pool: NHWC bf16 input")
        x = x.contiguous()  # the kernel indexes x as dense NHWC
        n, h, w, c = x.shape
        y = torch.empty(n, c, dtype=torch.bfloat16 if out_bf16 else torch.float32, device=x.device)
        N.check(N.lib().dca_ops_avgpool_fwd(N.ptr(x), N.ptr(y), n, h * w, c, int(out_bf16), N.stream(x.device)),
                "avgpool_fwd")
        ctx.shape = (n, h, w, c)
        return y

    @staticmethod
    def backward(ctx, dy):
        n, h, w, c = ctx.shape
        bf = dy.dtype == torch.bfloat16 and c % 8 == 0
        dy = dy.contiguous() if bf else dy.float().contiguous()
        dx = torch.empty(n, h, w, c, dtype=torch.bfloat16, device=dy.device)
        N.check(N.lib().dca_ops_avgpool_bwd(N.ptr(dy), N.ptr(dx), n, h * w, c, int(bf), N.stream(dy.device)),
                "avgpool_bwd")
        return dx, None


def global_avg_pool(x, out_dtype=torch.float32):
    """[N, H, W, C] bf16 -> [N, C] mean over H, W (fp32, or bf16: the fc GEMM operand without a cast pass)."""
    return _AvgPool.apply(x, out_dtype == torch.bfloat16)


# ------------------------------------------------------------------------------------------------------------
# Cross-entropy (mean) with the softmax gradient computed in the same kernel
# ------------------------------------------------------------------------------------------------------------
_TICKETS = {}


_TICKET_WORDS = 4096


def _ticket(dev, n: int = 1) -> torch.Tensor:
    """n consecutive zeroed device words for the in-launch "last workgroup" reductions (k_cross_entropy's mean, one
    per 64-column block of k_dy_prep's column sums).  The last workgroups reset them, so the words serve every
    launch of one stream in turn; handing them out round-robin from a ring of 4096 keeps launches that may overlap
    (other streams, graph replays) on different words."""
    assert 0 < n <= _TICKET_WORDS // 8, n
    ring = _TICKETS.get(dev)
    if ring is None:
        ring = _TICKETS[dev] = [torch.zeros(_TICKET_WORDS, dtype=torch.int32, device=dev), 0]
    if ring[1] + n > _TICKET_WORDS:
        ring[1] = 0
    start = ring[1]
    ring[1] += n
    return ring[0][start:start + n]


class _CrossEntropy(torch.autograd.Function):
    @staticmethod
    def forward(ctx, logits, labels):
        logits = logits.float().contiguous()
        B, K = logits.shape
        loss = torch.empty(B, dtype=torch.float32, device=logits.device)
        mean = torch.empty((), dtype=torch.float32, device=logits.device)
        dl = torch.empty_like(logits) if logits.requires_grad else None
        N.check(N.lib().dca_ops_cross_entropy(N.ptr(logits), N.ptr(labels.long().contiguous()), N.ptr(loss),
                                              N.ptr(dl), B, K, 1.0 / B, N.ptr(mean), N.ptr(_ticket(logits.device)),
                                              N.stream(logits.device)), "cross_entropy")
        ctx.save_for_backward(dl)
        return mean

    @staticmethod
    def backward(ctx, g):
        (dl,) = ctx.saved_tensors
        out = torch.empty_like(dl)
        g = g.float().contiguous()
        N.check(N.lib().dca_ops_scale_dev(N.ptr(dl), N.ptr(g), N.ptr(out), dl.numel(), N.stream(dl.device)),
                "scale_dev")
        return out, None


def cross_entropy(logits, labels):
    return _CrossEntropy.apply(logits, labels)


# ------------------------------------------------------------------------------------------------------------
# SGD over flat fp32 buffers (torch.optim.SGD semantics incl. momentum's first-step buffer init)
# ------------------------------------------------------------------------------------------------------------
def sgd_step_(p: torch.Tensor, g: torch.Tensor, lr: float, momentum: float = 0.0, weight_decay: float = 0.0,
              buf: Optional[torch.Tensor] = None, first: Optional[torch.Tensor] = None) -> None:
    _dev_check(p, g, buf)
    if p.dtype != torch.float32 or g.dtype != torch.float32 or not p.is_contiguous() or not g.is_contiguous():
        raise TypeError("sgd_step_: contiguous fp32 buffers")
    if momentum and buf is None:
        raise ValueError("sgd_step_: momentum needs a buffer")
    N.check(N.lib().dca_ops_sgd(N.ptr(p), N.ptr(g), N.ptr(buf), p.numel(), float(lr), float(momentum),
                                float(weight_decay), N.ptr(first), N.stream(p.device)), "sgd")
