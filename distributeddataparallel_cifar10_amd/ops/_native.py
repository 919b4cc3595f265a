"""ctypes binding of ``libdca_ops.so`` (csrc/ops_api.hip): raw launches on torch tensors and the current stream.

Loaded after ``import torch`` (one HIP runtime per process, see runtime/native.py).  There is no eager fallback
on a GPU: a missing library raises.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch

from .. import build as _build

ABI_VERSION = 13
_lock = threading.Lock()
_lib = None

c_void_p, c_int, c_long, c_float = ctypes.c_void_p, ctypes.c_int, ctypes.c_long, ctypes.c_float


class GemmArgs(ctypes.Structure):
    """Mirror of csrc/ops_gemm.hip::GemmArgs."""
    _fields_ = [
        ("A", c_void_p), ("B", c_void_p), ("C", c_void_p), ("bias", c_void_p), ("ws", c_void_p),
        ("M", c_int), ("N", c_int), ("K", c_int), ("lda", c_int), ("ldb", c_int), ("ldc", c_int),
        ("alpha", c_float), ("beta", c_float), ("ta", c_int), ("tb", c_int), ("fp8", c_int),
        ("relu", c_int), ("out_bf16", c_int), ("splits", c_int), ("k_per_split", c_int), ("alpha_dev", c_void_p),
        ("conv", c_int), ("cN", c_int), ("cH", c_int), ("cW", c_int), ("cC", c_int), ("cKH", c_int), ("cKW", c_int),
        ("cS", c_int), ("cP", c_int), ("cHo", c_int), ("cWo", c_int), ("col_stats", c_void_p),
        ("stats_shift", c_void_p), ("amax_a", c_void_p), ("amax_b", c_void_p),
        ("wperm_C", c_int), ("wperm_Cpad", c_int), ("wperm_T", c_int), ("single", c_int),
        ("stages", c_int), ("orow_S", c_int), ("orow_ph", c_int), ("orow_pw", c_int), ("orow_H", c_int),
        ("orow_W", c_int), ("orow_Ho", c_int), ("orow_Wo", c_int),
        ("beta_src", c_void_p), ("beta_mask", c_void_p),
    ]


class ConvGeom(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("N", "H", "W", "C", "KH", "KW", "stride", "pad", "Ho", "Wo", "K", "Kp")]


class PackDesc(ctypes.Structure):
    """Mirror of csrc/ops_nn.hip::PackDesc (one layer of the per-step weight pack)."""
    _fields_ = [("w", c_void_p), ("fwd", c_void_p), ("dgrad", c_void_p), ("q8", c_void_p), ("amax", c_void_p),
                ("co", c_int), ("ci", c_int), ("ci_pad", c_int), ("kh", c_int), ("kw", c_int), ("kp", c_int)]


class GatherDesc(ctypes.Structure):
    """Mirror of csrc/ops_nn.hip::GatherDesc."""
    _fields_ = [("w", c_void_p), ("idx", c_void_p), ("out", c_void_p), ("n", c_long)]


class PoolGeom(ctypes.Structure):
    _fields_ = [(n, c_int) for n in ("N", "H", "W", "C", "K", "S", "P", "Ho", "Wo")]


def _declare(lib):
    lib.dca_ops_last_error.restype = ctypes.c_char_p
    lib.dca_ops_abi_version.restype = c_int
    P = ctypes.POINTER
    lib.dca_ops_gemm.argtypes = [P(GemmArgs), c_void_p]
    lib.dca_ops_im2col.argtypes = [c_void_p, c_void_p, P(ConvGeom), c_void_p]
    lib.dca_ops_col2im.argtypes = [c_void_p, c_void_p, P(ConvGeom), c_int, c_void_p]
    lib.dca_ops_bn_fwd.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_long, c_int, c_float, c_float, c_int, c_int, c_void_p, c_void_p]
    lib.dca_ops_bn_fwd_parts.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p,
                                         c_void_p, c_void_p, c_long, c_int, c_float, c_float, c_int, c_int, c_void_p,
                                         c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                         c_void_p]
    lib.dca_ops_bn_eval.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                    c_long, c_int, c_float, c_int, c_int, c_void_p]
    lib.dca_ops_bn_bwd.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                   c_void_p, c_void_p, c_void_p, c_void_p, c_long, c_int, c_int, c_int, c_int,
                                   c_void_p, c_void_p, c_void_p]
    lib.dca_ops_maxpool_fwd.argtypes = [c_void_p, c_void_p, c_void_p, P(PoolGeom), c_void_p]
    lib.dca_ops_maxpool_bwd.argtypes = [c_void_p, c_void_p, c_void_p, P(PoolGeom), c_void_p]
    lib.dca_ops_bn_pool_fwd_parts.argtypes = [c_void_p, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                              c_void_p, c_float, c_float, c_void_p, c_void_p, P(PoolGeom), c_void_p,
                                              c_void_p]
    lib.dca_ops_bn_pool_bwd.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p, c_void_p,
                                        c_void_p, c_void_p, c_void_p, c_void_p, c_int, P(PoolGeom), c_void_p, c_void_p]
    lib.dca_ops_avgpool_fwd.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]
    lib.dca_ops_avgpool_bwd.argtypes = [c_void_p, c_void_p, c_int, c_int, c_int, c_int, c_void_p]
    lib.dca_ops_cross_entropy.argtypes = [c_void_p, c_void_p, c_void_p, c_void_p, c_int, c_int, c_float, c_void_p,
                                          c_void_p, c_void_p]
    lib.dca_ops_zero.argtypes = [c_void_p, ctypes.c_long, c_void_p]
    lib.dca_ops_scale_dev.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_long, c_void_p]
    lib.dca_ops_cast_bf16.argtypes = [c_void_p, c_void_p, ctypes.c_long, c_void_p]
    lib.dca_ops_add_i64.argtypes = [c_void_p, c_int, c_void_p]
    lib.dca_ops_dy_prep.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_void_p, c_void_p, c_void_p,
                                    ctypes.c_long, c_int, c_int, c_int, c_void_p]
    lib.dca_ops_gather_cols.argtypes = [c_void_p, c_int, c_void_p, c_int, c_void_p, c_int, c_int, c_void_p]
    lib.dca_ops_sgd.argtypes = [c_void_p, c_void_p, c_void_p, c_long, c_float, c_float, c_float, c_void_p, c_void_p]
    lib.dca_ops_quant_fp8.argtypes = [c_void_p, c_int, c_long, c_void_p, c_void_p, c_void_p]
    lib.dca_ops_fp8_alpha.argtypes = [c_void_p, c_void_p, c_float, c_void_p, c_void_p]
    lib.dca_ops_pack_weights.argtypes = [c_void_p, c_int, c_int, c_void_p, c_int, c_void_p]
    lib.dca_ops_pack_desc_size.restype = c_int
    lib.dca_ops_pack_gather.argtypes = [c_void_p, c_int, c_int, c_void_p]
    lib.dca_ops_gather_desc_size.restype = c_int
    lib.dca_ops_nchw_to_nhwc8.argtypes = [c_void_p, c_void_p, c_int, c_int, c_long, c_void_p]
    lib.dca_ops_nchw_to_s2d16.argtypes = [c_void_p, c_void_p] + [c_int] * 7 + [c_void_p]
    return lib


def library_path() -> str:
    return _build.lib_path("ops")


def lib():
    """The loaded ops library (built first if the sources changed); raises if it cannot be loaded."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        try:
            path = _build.build(variant="ops")
        except Exception as exc:  # toolchain missing: only acceptable if the .so already exists
            if not os.path.exists(path):
                raise RuntimeError(f"cannot build the ops library: {exc}") from exc
        handle = _declare(ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL))
        if handle.dca_ops_abi_version() != ABI_VERSION:
            raise RuntimeError(f"{path}: ABI {handle.dca_ops_abi_version()} != {ABI_VERSION} (stale build?)")
        if handle.dca_ops_pack_desc_size() != ctypes.sizeof(PackDesc) or \
                handle.dca_ops_gather_desc_size() != ctypes.sizeof(GatherDesc):
            raise RuntimeError(f"{path}: descriptor layout mismatch")
        _lib = handle
        return _lib


def check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib().dca_ops_last_error().decode(errors='replace')}")


def ptr(t):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def stream(device=None):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)
