"""ResNet-50 layer-1 3x3 convs at batch 256 (256x56x56x64 -> 64): forward (+ BN column statistics) and the implicit
weight gradient, event-timed; also the workload of the rocprofv3 --pmc runs in profiles/conv3x3_rows_r9.txt.

    python bench/conv3x3_64_bench.py [fwd|wgrad|both] [iters]
"""
import json
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402

which = sys.argv[1] if len(sys.argv) > 1 else "both"
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dev = torch.device("cuda", 0)
torch.manual_seed(0)
bf = torch.bfloat16
x = torch.randn(256, 56, 56, 64, device=dev).to(bf)
wt = torch.randn(64, 64, 3, 3, device=dev) * 0.05
geo = F._geom(x, wt, 1, 1)
wm = F._weight_matrix(wt, geo.K)
M = geo.N * geo.Ho * geo.Wo
shift = torch.zeros(64, device=dev)
parts = torch.zeros((M + 127) // 128, 64, 2, device=dev)
dy = torch.randn(M, 64, device=dev).to(bf)
sp = F._wgrad_splits(64, geo.K, M, True, row_w=56)
fns = {
    "fwd": lambda: F.gemm(x, wm, conv=1, geom=geo, mnk=(M, 64, geo.K), out_dtype=bf, col_stats=parts, stats_shift=shift),
    "wgrad": lambda: F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(64, geo.K, M), splits=sp),
}
for name, fn in fns.items():
    if which not in ("both", name):
        continue
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1e3 / iters
    print(json.dumps({"op": name, "us": round(us, 1), "tflops": round(2 * M * 64 * geo.K / us / 1e6, 1), "splits": sp}),
          flush=True)
