"""ResNet-50 stem conv (space-to-depth 4x4 over 16 channels, batch 256 at 224) bf16 + BN column statistics, event-timed.

    python bench/stem_conv_bench.py          (DCA_OPS_CONV_ROWS=0: the k_direct_conv<16, 4, 4> form)
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
shift = torch.zeros(64, device=dev)
parts = torch.zeros(((M + 127) // 128, 64, 2), device=dev)
fn = lambda: F.gemm(xs, e["fwd"], conv=1, geom=g, mnk=(M, 64, g.K), out_dtype=torch.bfloat16, col_stats=parts,  # noqa
                    stats_shift=shift)
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
print(json.dumps({"op": "stem_fwd", "us": round(us, 1), "tflops": round(2 * M * 64 * g.K / us / 1e6, 1)}))
