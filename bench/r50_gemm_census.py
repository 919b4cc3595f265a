"""Per-call GEMM census of one ResNet-50 ops-path training step: every ``functional.gemm`` call is timed
individually (device-synchronised events) and aggregated by shape / operand form, so GEMM work can be
prioritised by where the step's time actually goes.

    python bench/r50_gemm_census.py [--batch 64] [--fp8]      # JSON lines, largest total first
"""
from __future__ import annotations

import argparse
import collections
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--fp8", action="store_true")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    from distributeddataparallel_cifar10_amd.models.resnet50 import resnet50
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.ops import functional as F

    torch.manual_seed(0)
    model = OpsModel(resnet50().to(dev), fp8=a.fp8)
    x = torch.randn(a.batch, 3, 224, 224, device=dev)
    y = torch.randint(0, 1000, (a.batch,), device=dev)
    orig = F.gemm
    rec = collections.defaultdict(lambda: [0, 0.0, 0.0])
    active = [False]

    def timed(aa, bb, **kw):
        if not active[0]:
            return orig(aa, bb, **kw)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        out = orig(aa, bb, **kw)
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3
        if kw.get("conv"):
            M, Nn, K = kw["mnk"]
        else:
            M = aa.shape[1] if kw.get("ta") else aa.shape[0]
            K = aa.shape[0] if kw.get("ta") else aa.shape[1]
            Nn = bb.shape[1] if kw.get("tb") else bb.shape[0]
        kind = ("fp8 " if aa.dtype == torch.uint8 else "") + \
            {(0, 0, 0): "nt", (0, 1, 0): "dgrad(tb)", (1, 1, 0): "wgrad(ta,tb)", (0, 0, 1): "conv-fwd/dgrad",
             (1, 0, 2): "conv-wgrad"}.get((int(bool(kw.get("ta"))), int(bool(kw.get("tb"))), int(kw.get("conv", 0))), "other")
        key = (kind, M, Nn, K, kw.get("splits", 0))
        r = rec[key]
        r[0] += 1
        r[1] += us
        r[2] += 2.0 * M * Nn * K
        return out

    F.gemm = timed
    for _ in range(2):  # warm-up (allocator, fp8 delayed-scaling state)
        loss = cross_entropy(model(x), y)
        loss.backward()
    torch.cuda.synchronize()
    active[0] = True
    loss = cross_entropy(model(x), y)
    loss.backward()
    torch.cuda.synchronize()
    active[0] = False
    tot = sum(r[1] for r in rec.values())
    flop = sum(r[2] for r in rec.values())
    for key, (n, us, fl) in sorted(rec.items(), key=lambda kv: -kv[1][1]):
        print(json.dumps({"kind": key[0], "M": key[1], "N": key[2], "K": key[3], "splits": key[4], "calls": n,
                          "us": round(us, 1), "pct": round(100 * us / tot, 1), "tflops": round(fl / us / 1e6, 1)}))
    print(json.dumps({"total_gemm_us": round(tot, 1), "gemm_tflops": round(flop / tot / 1e6, 1),
                      "calls": sum(r[0] for r in rec.values())}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
