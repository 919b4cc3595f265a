"""Loader for the native engine library (ctypes, C ABI).

The library must be loaded AFTER ``import torch``: it links ``libamdhip64.so.7`` / ``librccl.so.1`` by SONAME and
so binds to the HIP runtime and RCCL that torch already mapped (one runtime per process).

On a machine with a GPU a missing or unloadable library is an error (``require_native``), never a silent fallback
to eager PyTorch ops.
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (must be imported before the native library, see module docstring)

from .. import build as _build

ABI_VERSION = 7  # csrc/engine.hip dca_abi_version(): DcaInit layout / C signatures
_lock = threading.Lock()
_lib = None


class NativeUnavailable(RuntimeError):
    pass


def _declare(lib):
    c_void_p, c_int, c_char_p = ctypes.c_void_p, ctypes.c_int, ctypes.c_char_p
    lib.dca_last_error.restype = c_char_p
    lib.dca_abi_version.restype = c_int
    lib.dca_nccl_unique_id.argtypes = [ctypes.c_char_p]
    lib.dca_engine_create.argtypes = [c_void_p, c_int, ctypes.POINTER(c_void_p)]
    lib.dca_engine_destroy.argtypes = [c_void_p]
    lib.dca_engine_derive.argtypes = [c_void_p]
    lib.dca_engine_set_indices.argtypes = [c_void_p, c_void_p, c_int]
    lib.dca_engine_set_cursor.argtypes = [c_void_p, c_int]
    lib.dca_engine_read_loss.argtypes = [c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(c_int), c_int]
    lib.dca_engine_run.argtypes = [c_void_p, c_int, c_int, c_int]
    lib.dca_engine_run_part.argtypes = [c_void_p, c_int, c_int]
    lib.dca_engine_run_checked.argtypes = [c_void_p, c_int, c_int, ctypes.POINTER(c_int)]
    lib.dca_engine_sync.argtypes = [c_void_p]
    lib.dca_engine_stream.argtypes = [c_void_p]
    lib.dca_engine_stream.restype = c_void_p
    lib.dca_engine_region.argtypes = [c_void_p, c_char_p]
    lib.dca_engine_region.restype = c_void_p
    lib.dca_engine_workspace_bytes.argtypes = [c_void_p]
    lib.dca_engine_workspace_bytes.restype = ctypes.c_size_t
    lib.dca_engine_ipc_handle.argtypes = [c_void_p, ctypes.c_char_p]
    lib.dca_engine_ipc_open.argtypes = [c_void_p, ctypes.c_char_p, c_int]
    lib.dca_engine_ipc_selftest.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.POINTER(c_int)]
    lib.dca_engine_ipc_selftest_fc.argtypes = [c_void_p, c_void_p, c_void_p, ctypes.c_float, ctypes.POINTER(c_int),
                                               ctypes.POINTER(c_int), ctypes.POINTER(c_int)]
    lib.dca_engine_ipc_bench.argtypes = [c_void_p, c_void_p, c_void_p, c_int, ctypes.POINTER(ctypes.c_float)]
    lib.dca_engine_errors.argtypes = [c_void_p, ctypes.POINTER(ctypes.c_uint), c_int]  # flags[2]
    lib.dca_engine_precapture.argtypes = [c_void_p, c_int]
    lib.dca_engine_kind.argtypes = [c_void_p]
    lib.dca_engine_set_shared_device.argtypes = [c_void_p, c_int]
    lib.dca_engine_set_epoch.argtypes = [c_void_p, c_int, c_int]
    lib.dca_engine_epoch.argtypes = [c_void_p, ctypes.POINTER(c_int)]
    lib.dca_engine_fc_in_step.argtypes = [c_void_p, c_int]
    lib.dca_engine_prologue.argtypes = [c_void_p, c_int]
    lib.dca_engine_comm_time.argtypes = [c_void_p, ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_longlong),
                                         c_int]
    return lib


def load_micro():
    """The calibration micro-benchmark library (bench/micro/engine_micro.hip; benchmarks only)."""
    path = _build.build(variant="micro")
    lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    c_int, fp, ip = ctypes.c_int, ctypes.POINTER(ctypes.c_float), ctypes.POINTER(ctypes.c_int)
    lib.dca_micro_last_error.restype = ctypes.c_char_p
    lib.dca_microbench_xgmi.argtypes = [c_int, c_int, fp, ip]
    lib.dca_microbench.argtypes = [c_int, c_int, c_int, c_int, fp]
    lib.dca_microbench_xchg.argtypes = [c_int, c_int, c_int, c_int, c_int, fp, ip]
    lib.dca_microbench_bnx.argtypes = [c_int, c_int, c_int, c_int, c_int, c_int, fp, ip]
    return lib


def variant() -> str:
    """Library variant selected by DCA_ENGINE_VARIANT ("" production, "stamps" diagnostic)."""
    return os.environ.get("DCA_ENGINE_VARIANT", "")


def library_path() -> str:
    return _build.lib_path(variant())


def load(build_if_missing: bool = True):
    """Return the loaded engine library (building it first if needed)."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        path = library_path()
        if build_if_missing:
            try:
                path = _build.build(variant=variant())
            except Exception as exc:  # toolchain missing: only acceptable if the .so already exists
                if not os.path.exists(path):
                    raise NativeUnavailable(f"cannot build native engine: {exc}") from exc
        if not os.path.exists(path):
            raise NativeUnavailable(f"native engine library not found at {path}")
        try:
            lib = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
        except OSError as exc:
            raise NativeUnavailable(f"cannot load {path}: {exc}") from exc
        _lib = _declare(lib)
        if _lib.dca_abi_version() != ABI_VERSION:
            _lib = None
            raise NativeUnavailable(f"{path}: ABI {lib.dca_abi_version()} != expected {ABI_VERSION} (stale build?)")
        return _lib


def require_native():
    """Load the engine or raise; used on every GPU code path (no silent eager fallback)."""
    return load(build_if_missing=True)


def last_error() -> str:
    return load(build_if_missing=False).dca_last_error().decode(errors="replace")


def check(rc: int, what: str):
    if rc != 0:
        lib = load(build_if_missing=False)
        raise RuntimeError(f"{what} failed: {lib.dca_last_error().decode(errors='replace')}")
