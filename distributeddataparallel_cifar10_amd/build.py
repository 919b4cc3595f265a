"""Build the native HIP/C++ code of the framework for gfx950 (MI355X), in-tree.

``python -m distributeddataparallel_cifar10_amd.build`` compiles, with ``hipcc --offload-arch=gfx950``:
  * ``csrc/engine.hip`` (the NetResDeep training engine + xGMI all-reduce) -> ``_lib/libdca_engine.so``
  * ``csrc/ops_api.hip`` (the general layer kernels of ``ops/``: MFMA GEMM bf16/fp8, im2col, BN, pooling, CE,
    SGD, fp8 quantisation) -> ``_lib/libdca_ops.so``
  * ``csrc/comm_api.hip`` (generic xGMI one-shot / two-shot all-reduce for any model's flat buckets)
    -> ``_lib/libdca_comm.so``
  * on request only (``build micro``): ``bench/micro/engine_micro.hip`` calibration kernels -> ``_lib/libdca_micro.so``
hipcc cross-compiles without
a GPU, so this runs on the CPU-only build host too.  The library links the HIP runtime and RCCL by SONAME
(``libamdhip64.so.7``, ``librccl.so.1``); loaded after ``import torch`` it binds to the copies torch already
loaded, so there is exactly one HIP runtime in the process.
"""
from __future__ import annotations

import hashlib
import os
import shutil
import subprocess
import sys

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(PKG_DIR, "csrc")
LIB_DIR = os.path.join(PKG_DIR, "_lib")
ENGINE_LIB = os.path.join(LIB_DIR, "libdca_engine.so")
OPS_LIB = os.path.join(LIB_DIR, "libdca_ops.so")
COMM_LIB = os.path.join(LIB_DIR, "libdca_comm.so")
MICRO_LIB = os.path.join(LIB_DIR, "libdca_micro.so")
_ENTRY = {"ops": ("ops_api.hip", OPS_LIB), "comm": ("comm_api.hip", COMM_LIB),
          # calibration micro-benchmarks (bench/micro): diagnostic, never loaded by the framework itself
          "micro": (os.path.join(os.path.dirname(PKG_DIR), "bench", "micro", "engine_micro.hip"), MICRO_LIB)}
ARCH = os.environ.get("DCA_OFFLOAD_ARCH", "gfx950")
# Variants: "" = production; "stamps" = diagnostic build with in-kernel phase stamps (-DDCA_STAMPS).
VARIANTS = {"": [], "stamps": ["-DDCA_STAMPS"], "ops": [], "comm": [], "micro": []}


def lib_path(variant: str = "") -> str:
    if variant in _ENTRY:
        return _ENTRY[variant][1]
    return ENGINE_LIB if not variant else os.path.join(LIB_DIR, f"libdca_engine_{variant}.so")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build the native engine)")


def _sources():
    return sorted(os.path.join(CSRC, f) for f in os.listdir(CSRC) if f.endswith((".hip", ".h", ".cpp")))


def _extra(variant: str) -> list:
    """Diagnostic builds only: extra hipcc flags from DCA_HIPCC_EXTRA (e.g. -DDCA_DETAIL_FWD=9 for the stamps)."""
    return os.environ.get("DCA_HIPCC_EXTRA", "").split() if variant == "stamps" else []


def _digest(variant: str = "") -> str:
    h = hashlib.sha256((ARCH + "|" + variant + "|" + " ".join(_extra(variant))).encode())
    extra = [_ENTRY["micro"][0]] if variant == "micro" else []
    for p in _sources() + extra:
        with open(p, "rb") as f:
            h.update(os.path.basename(p).encode())
            h.update(f.read())
    return h.hexdigest()


def build(force: bool = False, verbose: bool = False, variant: str = "") -> str:
    """Compile the engine library if sources changed; returns the .so path."""
    os.makedirs(LIB_DIR, exist_ok=True)
    out = lib_path(variant)
    stamp = out + ".sha256"
    digest = _digest(variant)
    if not force and os.path.exists(out) and os.path.exists(stamp):
        with open(stamp) as f:
            if f.read().strip() == digest:
                return out
    tmp = out + f".tmp{os.getpid()}"
    cmd = [
        _hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", "-shared",
        "-Wall", "-Wno-unused-function", "-Wno-unused-variable", *VARIANTS[variant], *_extra(variant),
        os.path.join(CSRC, _ENTRY[variant][0] if variant in _ENTRY else "engine.hip"), "-o", tmp,
        *([] if variant in _ENTRY else ["-lrccl"]),
    ]
    if verbose:
        print(" ".join(cmd), flush=True)
    res = subprocess.run(cmd, capture_output=True, text=True)
    if res.returncode != 0:
        raise RuntimeError(f"hipcc failed ({res.returncode}):\n{res.stderr[-6000:]}")
    os.replace(tmp, out)
    with open(stamp, "w") as f:
        f.write(digest)
    return out


def build_all(force: bool = False, verbose: bool = False, variants=("", "ops", "comm")) -> list:
    """Build the listed library variants (default: the engine, ops and comm libraries, compiled concurrently);
    returns their paths."""
    from concurrent.futures import ThreadPoolExecutor
    with ThreadPoolExecutor(max_workers=len(variants)) as ex:
        return list(ex.map(lambda v: build(force=force, verbose=verbose, variant=v), variants))


if __name__ == "__main__":
    wanted = [a for a in sys.argv[1:] if not a.startswith("--")]
    for v in wanted or (["", "ops", "comm", "stamps", "micro"] if "--all" in sys.argv else ["", "ops", "comm"]):
        print(build(force="--force" in sys.argv, verbose=True, variant=v))
