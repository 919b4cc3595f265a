"""GPU memory utilities (reference ``main.py:67-78`` ``free_gpu_cache``).

The reference prints GPU utilisation with GPUtil (nvidia-smi), empties the caching allocator and tears down the
device-0 context through numba.cuda; its only call site is commented out (``main.py:85``) and both GPUtil and
numba are hard import-time dependencies.  Neither exists for ROCm here, so:
  * utilisation comes from ``amd-smi`` (or ``rocm-smi``) when present, parsed loosely, never required;
  * ``torch.cuda.empty_cache()`` releases the HIP caching allocator's unused blocks;
  * there is no context teardown (destroying the HIP context under a live PyTorch runtime is unsafe).
"""
from __future__ import annotations

import json
import shutil
import subprocess
from typing import List

import torch


def gpu_usage() -> List[dict]:
    """[{gpu, busy_percent, vram_used_mb, vram_total_mb}] from amd-smi; [] if unavailable."""
    exe = shutil.which("amd-smi")
    if exe:
        try:
            out = subprocess.run([exe, "metric", "--usage", "--mem-usage", "--json"], capture_output=True, text=True,
                                 timeout=20)
            data = json.loads(out.stdout)
            rows = []
            for i, g in enumerate(data if isinstance(data, list) else data.get("gpu_data", [])):
                usage = g.get("usage", {}) or {}
                mem = g.get("mem_usage", {}) or {}

                def val(x):
                    return x.get("value") if isinstance(x, dict) else x
                rows.append({"gpu": g.get("gpu", i), "busy_percent": val(usage.get("gfx_activity")),
                             "vram_used_mb": val(mem.get("used_vram")), "vram_total_mb": val(mem.get("total_vram"))})
            return rows
        except Exception:
            return []
    return []


def show_utilization() -> None:
    rows = gpu_usage()
    if not rows:
        print("| GPU usage unavailable (amd-smi not found or not readable) |")
        return
    print("| ID | GPU % | MEM used (MB) | MEM total (MB) |")
    for r in rows:
        print(f"| {r['gpu']} | {r['busy_percent']} | {r['vram_used_mb']} | {r['vram_total_mb']} |")


def free_gpu_cache() -> None:
    print("Initial GPU Usage")
    show_utilization()
    if torch.cuda.is_available():
        torch.cuda.empty_cache()
    print("GPU Usage after emptying the cache")
    show_utilization()
