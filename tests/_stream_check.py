"""Run under DCA_OPS_STREAM=1 (tests/test_ops_gpu.py::test_gemm_stream_matches_torch): the persistent short-K GEMM
(csrc/ops_gemm.hip k_gemm_stream) against torch fp32 on plain NT shapes -- M tails, one to eight K-tiles, padded
row strides, bias, beta accumulation, the fused BN column statistics -- and the exact layout check (A = I).  One JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd import ops  # noqa: E402


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def main():
    assert os.environ.get("DCA_OPS_STREAM") == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    out = {}
    for M, N, K in [(128, 128, 64), (1000, 256, 64), (4097, 512, 128), (300, 1024, 256), (20000, 128, 512), (5000, 64, 128),
                    (70000, 256, 64)]:
        a = torch.randn(M, K, device=dev, generator=g).to(bf)
        b = (torch.randn(N, K, device=dev, generator=g) * torch.linspace(0.5, 2.0, K, device=dev)).to(bf)
        bias = torch.randn(N, device=dev, generator=g)
        ref = a.float() @ b.float().t()
        out[f"nt{M}x{N}x{K}_bf16"] = rel(ops.gemm(a, b, out_dtype=bf), ref)
        out[f"nt{M}x{N}x{K}_bf16_bias"] = rel(ops.gemm(a, b, bias=bias, out_dtype=bf), ref + bias)
        c0 = torch.randn(M, N, device=dev, generator=g).to(bf)
        c1 = c0.clone()
        ops.gemm(a, b, out_dtype=bf, out=c1, beta=1.0)
        out[f"nt{M}x{N}x{K}_beta"] = rel(c1, ref + c0.float())
        shift = torch.randn(N, device=dev, generator=g) * 0.1
        parts = torch.full(((M + 127) // 128, N, 2), float("nan"), device=dev)
        y = ops.gemm(a, b, out_dtype=bf, col_stats=parts, stats_shift=shift)
        d = y.float() - shift
        out[f"nt{M}x{N}x{K}_colstats"] = max(rel(parts[..., 0].sum(0), d.sum(0)),
                                             rel(parts[..., 1].sum(0), (d * d).sum(0)))
        out[f"nt{M}x{N}x{K}_colstats_y"] = rel(y, ref)
    # implicit convolutions (C % 64 == 0, N = 64 / 128): padding, stride 2, 1x1, M tails, BN statistics, beta
    from distributeddataparallel_cifar10_amd.ops import functional as F
    for n, h, c, co, k, st, pd in [(2, 14, 64, 64, 3, 1, 1), (3, 15, 128, 128, 3, 2, 1), (4, 9, 64, 128, 3, 1, 1),
                                   (2, 11, 128, 64, 1, 1, 0), (1, 57, 64, 64, 3, 1, 1)]:
        x = torch.randn(n, h, h, c, device=dev, generator=g).to(bf)
        wt = torch.randn(co, c, k, k, device=dev, generator=g) * 0.05
        geo = F._geom(x, wt, st, pd)
        wm = F._weight_matrix(wt, geo.K)
        Mc = geo.N * geo.Ho * geo.Wo
        ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), wt.to(bf).float(), stride=st, padding=pd)
        ref = ref.permute(0, 2, 3, 1).reshape(Mc, co)
        shift = torch.randn(co, device=dev, generator=g) * 0.1
        parts = torch.full(((Mc + 127) // 128, co, 2), float("nan"), device=dev)
        y = ops.gemm(x, wm, conv=1, geom=geo, mnk=(Mc, co, geo.K), out_dtype=bf, col_stats=parts, stats_shift=shift)
        tag = f"conv{n}x{h}x{c}->{co}_k{k}s{st}"
        out[tag] = rel(y, ref)
        d = y.float() - shift
        out[tag + "_colstats"] = max(rel(parts[..., 0].sum(0), d.sum(0)), rel(parts[..., 1].sum(0), (d * d).sum(0)))
        c0 = torch.randn(Mc, co, device=dev, generator=g).to(bf)
        c1 = c0.clone()
        ops.gemm(x, wm, conv=1, geom=geo, mnk=(Mc, co, geo.K), out_dtype=bf, out=c1, beta=1.0)
        out[tag + "_beta"] = rel(c1, ref + c0.float())
    # padded leading dimensions (views into wider buffers)
    a_w = torch.randn(3000, 192, device=dev, generator=g).to(bf)
    b_w = torch.randn(256, 136, device=dev, generator=g).to(bf)
    a, b = a_w[:, :128], b_w[:, :128]
    out["nt_strided"] = rel(ops.gemm(a, b, out_dtype=bf), a.float() @ b.float().t())
    # exact layout: C = I_M . B^T with small integers (bf16-exact)
    n = 256
    eye = torch.eye(n, device=dev, dtype=bf)
    bi = torch.arange(128 * n, device=dev).remainder(61).float().view(128, n).to(bf)  # B [N = 128, K = n]
    y = ops.gemm(eye, bi, out_dtype=bf)  # C[m, c] = B[c, m]
    out["identity_exact_err"] = float((y.float() - bi.float().t()).abs().max())
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
