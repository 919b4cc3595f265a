"""Run under DCA_OPS_PP=1 (tests/test_ops_gpu.py::test_gemm_pingpong_matches_torch): the ping-pong 256 x 256 GEMM
(csrc/ops_gemm.hip k_gemm_pp) against torch fp32 on plain NT shapes (tails in M, N and K), implicit 3x3 / 1x1
convolutions with C % 64 == 0 (padding, stride 2) and the fused BN column statistics.  Prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd import ops  # noqa: E402
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    assert os.environ.get("DCA_OPS_PP") == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    out = {}
    for M, N, K in [(256, 256, 256), (1000, 384, 520), (777, 130, 1000), (4096, 512, 2048), (2048, 128, 1152)]:
        a = torch.randn(M, K, device=dev, generator=g).to(bf)
        b = torch.randn(N, K, device=dev, generator=g).to(bf)
        bias = torch.randn(N, device=dev, generator=g)
        ref = a.float() @ b.float().t()
        out[f"nt{M}x{N}x{K}"] = rel(ops.gemm(a, b, out_dtype=torch.float32), ref)
        out[f"nt{M}x{N}x{K}_bf16_bias_relu"] = rel(ops.gemm(a, b, bias=bias, relu=True, out_dtype=bf),
                                                  torch.relu(ref + bias))
        shift = torch.randn(N, device=dev, generator=g) * 0.1
        parts = torch.empty((M + 127) // 128, N, 2, device=dev)
        y = ops.gemm(a, b, out_dtype=bf, col_stats=parts, stats_shift=shift)
        d = y.float() - shift
        out[f"nt{M}x{N}x{K}_colstats"] = max(rel(parts[..., 0].sum(0), d.sum(0)),
                                             rel(parts[..., 1].sum(0), (d * d).sum(0)))
    for n, h, c, co, k, s, p in [(4, 14, 64, 256, 3, 1, 1), (2, 15, 128, 128, 3, 2, 1), (8, 7, 512, 256, 3, 1, 1),
                                 (4, 9, 256, 320, 1, 1, 0)]:
        x = torch.randn(n, h, h, c, device=dev, generator=g).to(bf)
        w = torch.randn(co, c, k, k, device=dev, generator=g) * 0.05
        geo = F._geom(x, w, s, p)
        wm = F._weight_matrix(w, geo.K)
        Mc = geo.N * geo.Ho * geo.Wo
        y = ops.gemm(x, wm, conv=1, geom=geo, mnk=(Mc, co, geo.K), out_dtype=torch.float32)
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(bf).float(), stride=s, padding=p)
        out[f"conv{n}x{h}x{c}->{co}_k{k}s{s}"] = rel(y.view(n, geo.Ho, geo.Wo, co).permute(0, 3, 1, 2), ref)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
