"""Weight-gradient GEMMs of ResNet-50 at batch 256 (bf16, the shapes `functional._conv_bwd` issues), timed through
``functional.gemm`` exactly as the training step calls them (transposed-read kernel + split-K reduce into torch's
[Cout, Cin, KH, KW] fp32 layout), with a numerics check of every shape against a torch fp32 reference.

    python bench/wgrad_bench.py [--iters 20] [--only 3x3|1x1]      # one JSON line per shape
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402

# (n, h, w, cin, cout, k, stride, pad, calls) -- every distinct conv of ResNet-50 with its call count per step
SHAPES_3X3 = [
    (256, 56, 56, 64, 64, 3, 1, 1, 3),
    (256, 56, 56, 128, 128, 3, 2, 1, 1),
    (256, 28, 28, 128, 128, 3, 1, 1, 3),
    (256, 28, 28, 256, 256, 3, 2, 1, 1),
    (256, 14, 14, 256, 256, 3, 1, 1, 5),
    (256, 14, 14, 512, 512, 3, 2, 1, 1),
    (256, 7, 7, 512, 512, 3, 1, 1, 2),
    (256, 224, 224, 8, 64, 7, 2, 3, 1),
    (256, 56, 56, 256, 512, 1, 2, 0, 1),   # strided 1x1 downsamples: implicit-im2col B operand
    (256, 28, 28, 512, 1024, 1, 2, 0, 1),
    (256, 14, 14, 1024, 2048, 1, 2, 0, 1),
]
SHAPES_1X1 = [  # (pixels, cin, cout, calls)
    (802816, 64, 64, 1), (802816, 64, 256, 4), (802816, 256, 64, 2), (802816, 256, 128, 1),
    (200704, 128, 512, 4), (200704, 512, 128, 3), (200704, 512, 256, 1),
    (50176, 256, 1024, 6), (50176, 1024, 256, 5), (50176, 1024, 512, 1), (12544, 512, 2048, 3),
    (12544, 2048, 512, 2),
]


def timeit(fn, iters):
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


def check(dst, ref):
    err = (dst - ref).abs().max().item()
    scale = ref.abs().max().item()
    return err / max(scale, 1e-30)


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--only", default=None, choices=[None, "3x3", "1x1"])
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    tot_us = tot_fl = 0.0
    worst = 0.0
    if a.only in (None, "3x3"):
        for n, h, w, c, co, k, s, p, calls in SHAPES_3X3:
            x = torch.randn(n, h, w, c, device=dev).to(bf)
            wt = torch.empty(co, c, k, k, device=dev)
            g = F._geom(x, wt, s, p)
            M = g.N * g.Ho * g.Wo
            dy = (torch.randn(M, co, device=dev) * 0.1).to(bf)
            dst = torch.empty(co, c, k, k, device=dev)

            def run():
                F.gemm(dy, x, ta=True, conv=2, geom=g, mnk=(co, g.K, M), splits=F._wgrad_splits(co, g.K, M, True),
                       out=dst, beta=0.0, wperm=(c, g.C, k * k))
            us = timeit(run, a.iters)
            run()
            # reference on a slice of the batch (full-batch fp32 conv weight-gradient is slow and large)
            nb = max(1, n // 32)
            xs = x[:nb].permute(0, 3, 1, 2).float()
            dys = dy.view(n, g.Ho, g.Wo, co)[:nb].permute(0, 3, 1, 2).float()
            ref = torch.nn.grad.conv2d_weight(xs, wt.shape, dys, stride=s, padding=p)
            dst_s = torch.empty_like(dst)
            Ms = nb * g.Ho * g.Wo
            gs = F._geom(x[:nb].contiguous(), wt, s, p)
            F.gemm(dy[:Ms].contiguous(), x[:nb].contiguous(), ta=True, conv=2, geom=gs, mnk=(co, gs.K, Ms),
                   splits=F._wgrad_splits(co, gs.K, Ms, True), out=dst_s, beta=0.0, wperm=(c, gs.C, k * k))
            e = check(dst_s, ref)
            worst = max(worst, e)
            fl = 2.0 * M * co * k * k * c
            tot_us += us * calls
            tot_fl += fl * calls
            print(json.dumps({"kind": "conv-wgrad", "shape": f"{n}x{h}x{w}x{c}->{co} k{k}s{s}", "M": co,
                              "N": g.K, "K": M, "calls": calls, "us": round(us, 1),
                              "tflops": round(fl / us / 1e6, 1), "rel_err": float(f"{e:.2e}")}), flush=True)
    if a.only in (None, "1x1"):
        for P, c, co, calls in SHAPES_1X1:
            x = torch.randn(P, c, device=dev).to(bf)
            dy = (torch.randn(P, co, device=dev) * 0.1).to(bf)
            dst = torch.empty(co, c, 1, 1, device=dev)

            def run():
                F.gemm(dy, x, ta=True, tb=True, splits=F._wgrad_splits(co, c, P), out=dst, beta=0.0,
                       wperm=(c, c, 1))
            us = timeit(run, a.iters)
            run()
            ns = min(P, 8192)
            ref = dy[:ns].float().t() @ x[:ns].float()
            dst_s = torch.empty_like(dst)
            F.gemm(dy[:ns].contiguous(), x[:ns].contiguous(), ta=True, tb=True, splits=F._wgrad_splits(co, c, ns),
                   out=dst_s, beta=0.0, wperm=(c, c, 1))
            e = check(dst_s.view(co, c), ref)
            worst = max(worst, e)
            fl = 2.0 * P * co * c
            tot_us += us * calls
            tot_fl += fl * calls
            print(json.dumps({"kind": "wgrad", "shape": f"{P}x{c}->{co}", "M": co, "N": c, "K": P, "calls": calls,
                              "us": round(us, 1), "tflops": round(fl / us / 1e6, 1),
                              "gbps": round(2 * P * (c + co) / us / 1e3, 1), "rel_err": float(f"{e:.2e}")}),
                  flush=True)
    print(json.dumps({"total_us_per_step": round(tot_us, 1), "tflops": round(tot_fl / max(tot_us, 1e-9) / 1e6, 1),
                      "worst_rel_err": float(f"{worst:.2e}")}), flush=True)
    return 0 if worst < 2e-2 else 1


if __name__ == "__main__":
    sys.exit(main())
