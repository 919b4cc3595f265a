"""ResNet-50 3x3 / pad 1 convs at batch 256: layer 1 (56x56x64 -> 64, default) or layer 2 (--c 128: 28x28x128 ->
128): forward (+ BN column statistics) and the implicit weight gradient, event-timed; also the workload of the
rocprofv3 --pmc runs in profiles/conv3x3_rows_r9.txt.

    python bench/conv3x3_64_bench.py [fwd|wgrad|both] [iters] [--c 64|128]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("which", nargs="?", default="both", choices=["both", "fwd", "wgrad"])
ap.add_argument("iters", nargs="?", type=int, default=5)
ap.add_argument("--c", type=int, default=64, choices=[64, 128])
a = ap.parse_args()
c, hw = a.c, (56 if a.c == 64 else 28)
dev = torch.device("cuda", 0)
torch.manual_seed(0)
bf = torch.bfloat16
x = torch.randn(256, hw, hw, c, device=dev).to(bf)
wt = torch.randn(c, c, 3, 3, device=dev) * 0.05
geo = F._geom(x, wt, 1, 1)
wm = F._weight_matrix(wt, geo.K)
M = geo.N * geo.Ho * geo.Wo
shift = torch.zeros(c, device=dev)
parts = torch.zeros((M + 127) // 128, c, 2, device=dev)
dy = torch.randn(M, c, device=dev).to(bf)
sp = F._wgrad_splits(c, geo.K, M, True, row_w=hw)
fns = {
    "fwd": lambda: F.gemm(x, wm, conv=1, geom=geo, mnk=(M, c, geo.K), out_dtype=bf, col_stats=parts, stats_shift=shift),
    "wgrad": lambda: F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(c, geo.K, M), splits=sp),
}
for name, fn in fns.items():
    if a.which not in ("both", name):
        continue
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(a.iters):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / a.iters
    print(json.dumps({"op": name, "c": c, "us": round(us, 1), "tflops": round(2 * M * c * geo.K / us / 1e6, 1),
                      "splits": sp}), flush=True)
