"""Throughput of the ops-layer MFMA GEMM (csrc/ops_gemm.hip) on the shapes ResNet-50 (bs 64, 224^2) trains with.

    python bench/gemm_bench.py            # one JSON line per shape: us, TFLOP/s, GB/s (min traffic)
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd import ops  # noqa: E402
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402
from distributeddataparallel_cifar10_amd.ops import _native as N  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / iters


def main():
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    rows = []

    def rec(name, us, flop, bytes_):
        rows.append({"shape": name, "us": round(us, 1), "tflops": round(flop / us / 1e6, 1),
                     "gbps": round(bytes_ / us / 1e3, 1)})
        print(json.dumps(rows[-1]), flush=True)

    for M, Nn, K in [(4096, 4096, 4096), (200704, 64, 64), (200704, 256, 64), (50176, 128, 512), (200704, 128, 512),
                     (802816, 256, 64), (200704, 512, 128), (50176, 256, 1024),
                     (12544, 1024, 256), (3136, 2048, 512)]:
        a = torch.randn(M, K, device=dev).to(bf)
        b = torch.randn(Nn, K, device=dev).to(bf)
        us = timeit(lambda: ops.gemm(a, b, out_dtype=bf))
        rec(f"nt {M}x{Nn}x{K}", us, 2 * M * Nn * K, 2 * (M * K + Nn * K + M * Nn))
        qa, _ = ops.quantize_fp8(a)
        qb, _ = ops.quantize_fp8(b)
        if K % 16 == 0:
            us = timeit(lambda: ops.gemm(qa, qb, out_dtype=bf))
            rec(f"fp8 {M}x{Nn}x{K}", us, 2 * M * Nn * K, (M * K + Nn * K + 2 * M * Nn))
    # implicit 3x3 conv forward / wgrad / dgrad, layer1 and layer3 of ResNet-50 at bs 64
    for n, h, c, co in [(64, 56, 64, 64), (64, 14, 256, 256)]:
        x = torch.randn(n, h, h, c, device=dev).to(bf)
        w = torch.randn(co, c, 3, 3, device=dev) * 0.05
        g = F._geom(x, w, 1, 1)
        wm = F._weight_matrix(w, g.K)
        M = n * h * h
        fl = 2 * M * co * g.K
        us = timeit(lambda: ops.gemm(x, wm, conv=1, geom=g, mnk=(M, co, g.K), out_dtype=bf))
        rec(f"conv3x3 fwd {n}x{h}x{h}x{c}->{co}", us, fl, 2 * (M * c + M * co))
        dy = torch.randn(M, co, device=dev).to(bf)
        sp = F._wgrad_splits(co, g.K, M, True)
        us = timeit(lambda: ops.gemm(dy, x, ta=True, conv=2, geom=g, mnk=(co, g.K, M), splits=sp))
        rec(f"conv3x3 wgrad {n}x{h}x{h}x{c}->{co} splits {sp}", us, fl, 2 * (M * c + M * co))
        cols = torch.randn(M, g.K, device=dev).to(bf)
        us = timeit(lambda: ops.gemm(dy, cols, ta=True, tb=True, splits=sp))
        rec(f"explicit-cols wgrad {co}x{g.K}x{M} splits {sp}", us, fl, 2 * (M * g.K + M * co))


if __name__ == "__main__":
    main()
