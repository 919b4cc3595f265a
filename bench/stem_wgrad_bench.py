"""ResNet-50 stem weight gradient (s2d 4x4 over 16 channels, batch 256 at 224), incl. the split-K reduce, event-timed.

    python bench/stem_wgrad_bench.py          (DCA_OPS_WGRAD_ROWS=0: the k_wgrad form)
"""
import json
import os
import sys

import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402
dev = torch.device("cuda", 0)
torch.manual_seed(0)
conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(dev)
pack = F.WeightPack([conv], (), [conv])
pack.pack()
e = pack.get(conv)
x = torch.randn(256, 3, 224, 224, device=dev)
xs = F.nchw_to_s2d16(x)
wg, st, pd = F._s2d_args(conv.weight, 2, 3, e)
g = F._geom(xs, wg, st, pd)
M = g.N * g.Ho * g.Wo
dy = torch.randn(M, 64, device=dev).to(torch.bfloat16)
d4 = torch.empty(64, 16, 4, 4, device=dev)
sp = F._wgrad_splits(64, g.K, M, True, row_w=g.W)
fn = lambda: F.gemm(dy, xs, ta=True, conv=2, geom=g, mnk=(64, g.K, M), splits=sp, out=d4, wperm=(16, 16, 16))  # noqa
for _ in range(3):
    fn()
torch.cuda.synchronize()
a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
a.record()
for _ in range(20):
    fn()
b.record()
torch.cuda.synchronize()
us = a.elapsed_time(b) * 1e3 / 20
print(json.dumps({"op": "stem_wgrad", "us": round(us, 1), "tflops": round(2 * M * 64 * g.K / us / 1e6, 1), "splits": sp}))
