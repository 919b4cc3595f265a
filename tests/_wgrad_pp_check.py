"""Run under DCA_OPS_WGRAD_PP_ALL=1 (tests/test_ops_gpu.py::test_wgrad_pingpong_all_forms): every form of the
ping-pong weight-gradient kernel (csrc/ops_wgrad.hip k_wgrad_pp), including the ones its shape rule leaves on
k_wgrad -- the 64-wide column tile and the swapped implicit-im2col row side -- against torch fp32 on plain and
implicit-conv shapes with ragged tails.  Prints one JSON line of relative errors."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd import ops  # noqa: E402
from distributeddataparallel_cifar10_amd.ops import functional as F  # noqa: E402


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30))


def main():
    assert os.environ.get("DCA_OPS_WGRAD_PP_ALL") == "1"
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(0)
    bf = torch.bfloat16
    out = {}
    for M, N, K, sp in [(256, 64, 4096, 4), (64, 576, 5000, 8), (64, 264, 777, 1), (128, 1152, 3000, 5),
                        (264, 72, 999, 3)]:
        a = torch.randn(K, M, device=dev, generator=g).to(bf)
        b = (torch.randn(K, N, device=dev, generator=g) * torch.linspace(0.5, 2.0, N, device=dev)).to(bf)
        out[f"wgrad{M}x{N}x{K}"] = rel(ops.gemm(a, b, ta=True, tb=True, splits=sp), a.float().t() @ b.float())
    for n, h, c, co, k, s, p in [(3, 14, 64, 64, 3, 1, 1), (2, 15, 128, 128, 3, 2, 1), (2, 20, 8, 64, 7, 2, 3),
                                 (2, 13, 64, 256, 3, 1, 1)]:
        x = torch.randn(n, h, h, c, device=dev, generator=g).to(bf)
        w = torch.empty(co, c, k, k, device=dev)
        geo = F._geom(x, w, s, p)
        M = n * geo.Ho * geo.Wo
        dy = torch.randn(M, co, device=dev, generator=g).to(bf)
        ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), w.shape,
                                          dy.float().view(n, geo.Ho, geo.Wo, co).permute(0, 3, 1, 2), stride=s,
                                          padding=p)
        o = torch.empty_like(w)
        F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(co, geo.K, M), splits=F._wgrad_splits(co, geo.K, M), out=o,
               wperm=(c, c, k * k))
        out[f"conv{n}x{h}x{c}->{co}k{k}s{s}"] = rel(o, ref)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
