"""Phase ranges for profilers: one context manager that opens a torch.profiler range and a roctx
range (``rocprofv3 --marker-trace`` shows it on the HIP timeline).

The roctx library (``libroctx64.so`` or the rocprofiler-sdk one) is loaded lazily with ctypes; where it is
absent the roctx half is a no-op, so the training loop never depends on it.
"""
from __future__ import annotations

import ctypes
import os
from contextlib import contextmanager

from torch.profiler import record_function

_ROCTX = None
_TRIED = False


def _roctx():
    global _ROCTX, _TRIED
    if not _TRIED:
        _TRIED = True
        for name in ("libroctx64.so", "librocprofiler-sdk-roctx.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(name)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                _ROCTX = lib
                break
            except OSError:
                continue
    return _ROCTX


def roctx_available() -> bool:
    return _roctx() is not None and os.environ.get("DCA_NO_ROCTX") != "1"


@contextmanager
def trace_range(name: str):
    """``with trace_range("forward"): ...`` -- torch.profiler + roctx range."""
    lib = _roctx() if os.environ.get("DCA_NO_ROCTX") != "1" else None
    if lib is not None:
        lib.roctxRangePushA(name.encode())
    try:
        with record_function(name):
            yield
    finally:
        if lib is not None:
            lib.roctxRangePop()
