"""Short-K / wide-output GEMMs of ResNet-50 at batch 256 (the 1x1 expand / reduce convolutions and their dgrads):
time per call with the fused BatchNorm column statistics the forward uses, against the HBM floor of the call
(A read once + C written once).

    python bench/gemm_shortk.py [--no-stats]        # one JSON line per shape
Dispatch knobs (DCA_OPS_*) are read once per process, so A/B runs use one process per setting.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd import ops  # noqa: E402

SHAPES = [(802816, 256, 64), (50176, 1024, 256), (200704, 512, 128), (802816, 64, 256), (200704, 128, 512),
          (12544, 2048, 512), (50176, 256, 1024), (802816, 128, 256)]


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
    ap = argparse.ArgumentParser()
    ap.add_argument("--no-stats", action="store_true")
    ap.add_argument("--tag", default=os.environ.get("DCA_TAG", "default"))
    ap.add_argument("--shape", default=None, help="MxNxK: only this shape")
    ap.add_argument("--beta", action="store_true", help="accumulate into the output (C += A B^T), no statistics")
    ap.add_argument("--library", action="store_true",
                    help="also time the library path on the same operands: torch.matmul (hipBLASLt) / torch conv2d "
                         "(MIOpen, channels-last), no statistics")
    ap.add_argument("--conv", default=None,
                    help="NxHxCxCO[xKxSxP]: an implicit convolution forward instead (default 3x3, stride 1, pad 1)")
    a = ap.parse_args()
    shapes = [tuple(int(v) for v in a.shape.split("x"))] if a.shape else SHAPES
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    if a.conv:
        from distributeddataparallel_cifar10_amd.ops import functional as F
        v = [int(t) for t in a.conv.split("x")]
        n, h, c, co = v[:4]
        kk, st, pd = v[4:7] if len(v) >= 7 else (3, 1, 1)
        x = torch.randn(n, h, h, c, device=dev).to(bf)
        wt = torch.randn(co, c, kk, kk, device=dev) * 0.05
        geo = F._geom(x, wt, st, pd)
        wm = F._weight_matrix(wt, geo.K)
        M = n * geo.Ho * geo.Wo
        kw = dict(col_stats=torch.zeros((M + 127) // 128, co, 2, device=dev), stats_shift=torch.zeros(co, device=dev))
        us = timeit(lambda: ops.gemm(x, wm, conv=1, geom=geo, mnk=(M, co, geo.K), out_dtype=bf, **kw))
        print(json.dumps({"tag": a.tag, "conv3x3": a.conv, "us": round(us, 1),
                          "tflops": round(2 * M * co * geo.K / us / 1e6, 1)}), flush=True)
        if a.library:
            xn = x.permute(0, 3, 1, 2)  # NCHW view of the NHWC tensor: channels-last for MIOpen
            wn = wt.to(bf).contiguous(memory_format=torch.channels_last)
            us = timeit(lambda: torch.nn.functional.conv2d(xn, wn, stride=st, padding=pd))
            print(json.dumps({"tag": "library", "conv3x3": a.conv, "us": round(us, 1),
                              "tflops": round(2 * M * co * geo.K / us / 1e6, 1)}), flush=True)
        return
    for M, N, K in shapes:
        x = torch.randn(M, K, device=dev).to(bf)
        w = torch.randn(N, K, device=dev).to(bf)
        kw = {}
        if a.beta:
            kw = dict(out=torch.zeros(M, N, device=dev, dtype=bf), beta=1.0)
        elif not a.no_stats:
            kw = dict(col_stats=torch.zeros((M + 127) // 128, N, 2, device=dev),
                      stats_shift=torch.zeros(N, device=dev))
        y = ops.gemm(x, w, out_dtype=bf, **kw)
        ref = (x.float() @ w.float().t())
        err = ((y.float() - ref).norm() / ref.norm()).item()
        us = timeit(lambda: ops.gemm(x, w, out_dtype=bf, **kw))
        floor_us = 2 * (M * K + M * N) / 5.0e6  # at 5 TB/s
        print(json.dumps({"tag": a.tag, "shape": f"{M}x{N}x{K}", "stats": not a.no_stats and not a.beta, "beta": a.beta, "us": round(us, 1),
                          "tflops": round(2 * M * N * K / us / 1e6, 1),
                          "gbps": round(2 * (M * K + (2 if a.beta else 1) * M * N) / us / 1e3, 1), "floor_us_5tbs": round(floor_us, 1),
                          "rel_err": round(err, 5)}), flush=True)
        if a.library:
            us = timeit(lambda: torch.matmul(x, w.t()))
            print(json.dumps({"tag": "library", "shape": f"{M}x{N}x{K}", "us": round(us, 1),
                              "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)
        del x, w, y, ref


if __name__ == "__main__":
    main()
