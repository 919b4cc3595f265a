"""Unit tests of the ops-layer HIP kernels (csrc/ops_*.hip) against plain PyTorch fp32 references of the same op
(layer 1: one test family per kernel family, random + ragged shapes, asymmetric operands)."""
import os

import pytest
import torch
import torch.nn.functional as TF

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def _bf(x):
    return x.to(torch.bfloat16)


@pytest.mark.parametrize("M,N,K,ta,tb", [(256, 128, 64, 0, 0), (300, 200, 136, 0, 0), (77, 10, 32, 0, 0),
                                         (130, 96, 200, 0, 1), (64, 48, 1000, 1, 1), (10, 32, 37, 1, 1),
                                         (512, 256, 4096, 0, 0)])
def test_gemm_bf16(gpu, M, N, K, ta, tb):
    from distributeddataparallel_cifar10_amd.ops import gemm
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N)
    a = torch.randn(M, K, device=gpu, generator=g)
    b = torch.randn(N, K, device=gpu, generator=g) * torch.linspace(0.5, 2.0, K, device=gpu)  # asymmetric B
    bias = torch.randn(N, device=gpu, generator=g)
    A = _bf(a.t().contiguous() if ta else a)
    B = _bf(b.t().contiguous() if tb else b)
    ref = _bf(a).float() @ _bf(b).float().t() + bias
    out = gemm(A, B, ta=bool(ta), tb=bool(tb), bias=bias)
    assert _rel(out, ref) < 1e-5, _rel(out, ref)
    out2 = gemm(A, B, ta=bool(ta), tb=bool(tb), bias=bias, relu=True, out_dtype=torch.bfloat16, splits=3)
    assert _rel(out2.float(), ref.clamp_min(0)) < 1e-2


def test_gemm_pingpong_matches_torch(gpu):
    """The ping-pong 256 x 256 GEMMs on shapes the production rule routes to them (N % 256 == 0, >= 160 output
    tiles): k_gemm_pp4 (K % 64 == 0, K >= 512) and k_gemm_pp (K = 1040: K % 64 != 0, K >= 1024); plain NT with M / K
    tails, bf16 output + bias + ReLU, the fused BN column statistics, and an implicit 3x3 convolution with C % 64 == 0
    -- against torch fp32."""
    from distributeddataparallel_cifar10_amd import ops
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(0)
    bf = torch.bfloat16
    for M, N, K in [(4096, 2560, 1024), (4000, 2560, 1040), (4000, 2560, 576)]:
        a = torch.randn(M, K, device=gpu, generator=g).to(bf)
        b = torch.randn(N, K, device=gpu, generator=g).to(bf)
        bias = torch.randn(N, device=gpu, generator=g)
        ref = a.float() @ b.float().t()
        assert _rel(ops.gemm(a, b, out_dtype=torch.float32), ref) < 2e-3
        assert _rel(ops.gemm(a, b, bias=bias, relu=True, out_dtype=bf).float(), torch.relu(ref + bias)) < 1e-2
        shift = torch.randn(N, device=gpu, generator=g) * 0.1
        parts = torch.empty((M + 127) // 128, N, 2, device=gpu)
        y = ops.gemm(a, b, out_dtype=bf, col_stats=parts, stats_shift=shift)
        d = y.float() - shift
        assert _rel(parts[..., 0].sum(0), d.sum(0)) < 1e-2 and _rel(parts[..., 1].sum(0), (d * d).sum(0)) < 1e-2
    x = torch.randn(64, 26, 26, 128, device=gpu, generator=g).to(bf)  # 43264 x 256 x 1152: 169 tiles
    w = torch.randn(256, 128, 3, 3, device=gpu, generator=g) * 0.05
    geo = F._geom(x, w, 1, 1)
    wm = F._weight_matrix(w, geo.K)
    Mc = geo.N * geo.Ho * geo.Wo
    y = ops.gemm(x, wm, conv=1, geom=geo, mnk=(Mc, 256, geo.K), out_dtype=torch.float32)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), w.to(bf).float(), padding=1)
    assert _rel(y.view(64, 26, 26, 256).permute(0, 3, 1, 2), ref) < 2e-3


def test_gemm_256_exact_integers(gpu):
    """The 256 x 256 GEMM (k_gemm_pp4, the production route of these shapes) on small-integer bf16 operands, where
    fp32 accumulation is exact: plain NT with an M tail and padded rows, and an implicit 3x3 convolution with padding
    taps -- bitwise against float64 references (catches any staging, swizzle, buffer or fragment-layout error
    exactly)."""
    from distributeddataparallel_cifar10_amd import ops
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(5)
    bf = torch.bfloat16
    for M, N, K, lda in [(4096, 2560, 1024, 1024), (4000, 2560, 2048, 2056), (4096, 4096, 4096, 4096)]:
        a = torch.randint(-3, 4, (M, lda), device=gpu, generator=g).to(bf)[:, :K]
        b = torch.randint(-3, 4, (N, K), device=gpu, generator=g).to(bf)
        ref = (a.double() @ b.double().t()).float()
        out = ops.gemm(a, b, out_dtype=torch.float32)
        assert torch.equal(out, ref), (M, N, K, (out - ref).abs().max().item())
    x = torch.randint(-2, 3, (64, 26, 26, 128), device=gpu, generator=g).to(bf)  # 43264 x 256 x 1152: 169 tiles
    w = torch.randint(-2, 3, (256, 128, 3, 3), device=gpu, generator=g).float()
    geo = F._geom(x, w, 1, 1)
    wm = F._weight_matrix(w, geo.K)
    y = ops.gemm(x, wm, conv=1, geom=geo, mnk=(geo.N * geo.Ho * geo.Wo, 256, geo.K), out_dtype=torch.float32)
    ref = torch.nn.functional.conv2d(x.double().permute(0, 3, 1, 2), w.double(), padding=1).float()
    assert torch.equal(y.view(64, 26, 26, 256).permute(0, 3, 1, 2), ref)


def test_gemm_stream_matches_torch(gpu):
    """The persistent short-K GEMM (DCA_OPS_STREAM=1, read once per process: run in a child) on plain NT shapes
    with M tails, 1-8 K-tiles, padded strides, bias, beta and the fused BN column statistics (the 128 x 128 tiles
    store through the LDS output image), against torch fp32; plus an exact layout check (A = I)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "tests", "_stream_check.py")], capture_output=True,
                       text=True, env=dict(os.environ, DCA_OPS_STREAM="1"), timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert res.pop("identity_exact_err") == 0.0, res
    bad = {k: v for k, v in res.items() if not v <= 1e-2}
    assert not bad, (bad, res)


def test_gemm_identity_layout(gpu):
    """A = I with an asymmetric B must return B^T exactly (catches row/col swaps in the C write)."""
    from distributeddataparallel_cifar10_amd.ops import gemm
    n = 64
    a = torch.eye(n, device=gpu, dtype=torch.bfloat16)
    b = torch.arange(n * n, device=gpu, dtype=torch.float32).remainder(97).view(n, n).to(torch.bfloat16)
    out = gemm(a, b)  # C[m, n] = sum_k I[m,k] B[n,k] = B[n, m]
    assert torch.equal(out, b.float().t())


def test_gemm_fp8_exact_integers(gpu):
    """fp8 e4m3 operands holding small integers (exactly representable) give exact products."""
    from distributeddataparallel_cifar10_amd.ops import gemm
    M, N, K = 160, 144, 256
    g = torch.Generator(device=gpu).manual_seed(3)
    a = torch.randint(-4, 5, (M, K), device=gpu, generator=g).float()
    b = torch.randint(-4, 5, (N, K), device=gpu, generator=g).float()
    qa = a.to(torch.float8_e4m3fn).view(torch.uint8)
    qb = b.to(torch.float8_e4m3fn).view(torch.uint8)
    out = gemm(qa, qb)
    assert torch.equal(out, a @ b.t())


def test_quantize_fp8_and_scaled_gemm(gpu):
    from distributeddataparallel_cifar10_amd.ops import fp8_alpha, gemm, quantize_fp8
    g = torch.Generator(device=gpu).manual_seed(4)
    x = torch.randn(512, 256, device=gpu, generator=g)
    w = torch.randn(384, 256, device=gpu, generator=g) * 0.05
    qx, ax = quantize_fp8(_bf(x))
    qw, aw = quantize_fp8(w)
    amax = ax.view(torch.float32).item()
    assert abs(amax - _bf(x).float().abs().max().item()) < 1e-6
    deq = qx.view(torch.float8_e4m3fn).float() * amax / 448.0
    assert _rel(deq, _bf(x).float()) < 0.05
    out = gemm(qx, qw, alpha_dev=fp8_alpha(ax, aw))
    assert _rel(out, x @ w.t()) < 0.06


@pytest.mark.parametrize("n,h,c,co,k,s,p,bias", [(2, 16, 32, 32, 3, 1, 1, False), (3, 32, 3, 32, 3, 1, 1, True),
                                                  (2, 14, 16, 24, 7, 2, 3, False), (2, 9, 64, 48, 1, 2, 0, False),
                                                  (4, 8, 64, 128, 1, 1, 0, False), (2, 10, 3, 16, 3, 2, 1, False),
                                                  # C % 64 == 0 3x3: the implicit-conv buffer-load fast path (padding
                                                  # taps, a partial last M tile; stride 1 dgrad runs it too)
                                                  (2, 12, 64, 64, 3, 1, 1, False), (2, 13, 128, 64, 3, 2, 1, False)])
def test_conv2d_fwd_bwd(gpu, n, h, c, co, k, s, p, bias):
    from distributeddataparallel_cifar10_amd.ops import conv2d
    g = torch.Generator(device=gpu).manual_seed(n * h + c)
    x = _bf(torch.randn(n, h, h, c, device=gpu, generator=g)).requires_grad_()
    w = (torch.randn(co, c, k, k, device=gpu, generator=g) * 0.2).requires_grad_()
    b = torch.randn(co, device=gpu, generator=g).requires_grad_() if bias else None
    y = conv2d(x, w, b, stride=s, pad=p)
    dy = torch.randn(y.shape, device=gpu, generator=g)
    y.backward(_bf(dy))
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    wr = _bf(w.detach()).float().requires_grad_()
    br = b.detach().clone().requires_grad_() if bias else None
    yr = TF.conv2d(xr, wr, br, stride=s, padding=p)
    yr.backward(_bf(dy).float().permute(0, 3, 1, 2))
    assert _rel(y.float().permute(0, 3, 1, 2), yr) < 1e-2
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 2e-2
    assert _rel(w.grad, wr.grad) < 1e-2
    if bias:
        assert _rel(b.grad, br.grad) < 1e-2


@pytest.mark.parametrize("res_mode,relu", [(0, True), (1, True), (2, True), (0, False)])
def test_batch_norm_act(gpu, res_mode, relu):
    from distributeddataparallel_cifar10_amd.ops import batch_norm_act
    g = torch.Generator(device=gpu).manual_seed(res_mode * 2 + relu)
    n, h, c = 4, 12, 48
    x = _bf(torch.randn(n, h, h, c, device=gpu, generator=g) * 2 + 0.5).requires_grad_()
    r = _bf(torch.randn(n, h, h, c, device=gpu, generator=g)).requires_grad_() if res_mode else None
    bn = torch.nn.BatchNorm2d(c).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    ref_bn = torch.nn.BatchNorm2d(c).to(gpu)
    ref_bn.load_state_dict(bn.state_dict())
    y = batch_norm_act(x, bn, r=r, relu=relu, res_mode=res_mode)
    dy = torch.randn(y.shape, device=gpu, generator=g)
    y.backward(_bf(dy))
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    rr = r.detach().float().permute(0, 3, 1, 2).requires_grad_() if res_mode else None
    z = ref_bn(xr)
    if res_mode == 2:
        z = z + rr
    if relu:
        z = torch.relu(z)
    if res_mode == 1:
        z = z + rr
    z.backward(_bf(dy).float().permute(0, 3, 1, 2))
    assert _rel(y.float().permute(0, 3, 1, 2), z) < 1e-2
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 2e-2
    assert _rel(bn.weight.grad, ref_bn.weight.grad) < 1e-3
    assert _rel(bn.bias.grad, ref_bn.bias.grad) < 1e-3
    if res_mode:
        assert _rel(r.grad.float().permute(0, 3, 1, 2), rr.grad) < 1e-2
    assert _rel(bn.running_mean, ref_bn.running_mean) < 1e-5
    assert _rel(bn.running_var, ref_bn.running_var) < 1e-5
    assert int(bn.num_batches_tracked) == int(ref_bn.num_batches_tracked) == 1


@pytest.mark.parametrize("n,h,c", [(8, 64, 64), (16, 96, 136), (32, 320, 8), (2, 48, 1024)])
def test_batch_norm_partial_reduction_shapes(gpu, n, h, c):
    """The ticketed partial-row reduction (k_bn_fin_ticket) of the BN statistics / backward sums on shapes with many
    partial rows (up to 12,800: several rows per workgroup and up to 100 row sums per column block), a partial last
    64-channel column block (C = 136, 8) and many column blocks (C = 1024): output, running statistics and
    dgamma / dbeta against torch fp32; a second call reuses the ticket words the first one reset."""
    from distributeddataparallel_cifar10_amd.ops import batch_norm_act
    g = torch.Generator(device=gpu).manual_seed(n + h + c)
    bn = torch.nn.BatchNorm2d(c).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    ref_bn = torch.nn.BatchNorm2d(c).to(gpu)
    ref_bn.load_state_dict(bn.state_dict())
    for it in range(2):
        x = _bf(torch.randn(n, h, h, c, device=gpu, generator=g) * 2 + 0.5 + it).requires_grad_()
        bn.zero_grad()
        ref_bn.zero_grad()
        y = batch_norm_act(x, bn, relu=True)
        dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
        y.backward(dy)
        xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
        z = torch.relu(ref_bn(xr))
        z.backward(dy.float().permute(0, 3, 1, 2))
        assert _rel(y.float().permute(0, 3, 1, 2), z) < 1e-2
        assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 2e-2
        assert _rel(bn.weight.grad, ref_bn.weight.grad) < 1e-3
        assert _rel(bn.bias.grad, ref_bn.bias.grad) < 1e-3
        assert _rel(bn.running_mean, ref_bn.running_mean) < 1e-5
        assert _rel(bn.running_var, ref_bn.running_var) < 1e-5


# (3, 2, 1, even h) with c % 8 == 0 takes the output-driven k_maxpool_bwd_k3s2 backward (h = 14: odd Ho edge)
@pytest.mark.parametrize("k,s,p,h", [(2, 2, 0, 16), (3, 2, 1, 15), (2, 2, 0, 7), (3, 2, 1, 16), (3, 2, 1, 14)])
@pytest.mark.parametrize("c", [24, 5])
def test_max_pool(gpu, k, s, p, h, c):
    from distributeddataparallel_cifar10_amd.ops import max_pool2d
    g = torch.Generator(device=gpu).manual_seed(k + h)
    x = _bf(torch.randn(2, h, h, c, device=gpu, generator=g)).requires_grad_()
    y = max_pool2d(x, k, s, p)
    dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = TF.max_pool2d(xr, k, s, p)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert torch.equal(y.float().permute(0, 3, 1, 2), yr)
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 1e-2


def test_max_pool_resnet_stem_shape(gpu):
    """The ResNet stem pool (3x3/2/1, 112 -> 56, 64 channels) through the output-driven backward."""
    from distributeddataparallel_cifar10_amd.ops import max_pool2d
    g = torch.Generator(device=gpu).manual_seed(5)
    x = _bf(torch.randn(3, 112, 112, 64, device=gpu, generator=g)).requires_grad_()
    y = max_pool2d(x, 3, 2, 1)
    dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    yr = TF.max_pool2d(xr, 3, 2, 1)
    yr.backward(dy.float().permute(0, 3, 1, 2))
    assert torch.equal(y.float().permute(0, 3, 1, 2), yr)
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 1e-2


def test_avg_pool_and_cross_entropy(gpu):
    from distributeddataparallel_cifar10_amd.ops import cross_entropy, global_avg_pool
    g = torch.Generator(device=gpu).manual_seed(9)
    x = _bf(torch.randn(5, 7, 7, 40, device=gpu, generator=g)).requires_grad_()
    y = global_avg_pool(x)
    y.backward(torch.ones_like(y))
    assert _rel(y, x.detach().float().mean((1, 2))) < 1e-5
    assert _rel(x.grad.float(), torch.full_like(x.grad.float(), 1 / 49)) < 1e-2
    logits = (torch.randn(33, 1000, device=gpu, generator=g) * 3).requires_grad_()
    labels = torch.randint(0, 1000, (33,), device=gpu, generator=g)
    loss = cross_entropy(logits, labels)
    loss.backward()
    lr_ = logits.detach().clone().requires_grad_()
    ref = TF.cross_entropy(lr_, labels)
    ref.backward()
    assert abs(loss.item() - ref.item()) < 1e-4
    assert _rel(logits.grad, lr_.grad) < 1e-4


@pytest.mark.parametrize("R,N,dyt,yt", [(256, 1000, torch.float32, torch.float32), (33, 10, torch.float32, None),
                                         (5000, 64, torch.bfloat16, torch.bfloat16), (1, 130, torch.bfloat16, None),
                                         (2048, 2048, torch.float32, torch.bfloat16), (70000, 24, torch.bfloat16, None)])
def test_dy_prep(gpu, R, N, dyt, yt):
    """k_dy_prep (2-D grid, per-column-block tickets): masked bf16 operand and bias gradient, plain and accumulated
    into a sink, repeated launches (tickets reset by the last blocks)."""
    from distributeddataparallel_cifar10_amd.ops.functional import dy_prep
    g = torch.Generator(device=gpu).manual_seed(R + N)
    dy = torch.randn(R, N, device=gpu, generator=g).to(dyt)
    y = torch.randn(R, N, device=gpu, generator=g).to(yt) if yt is not None else None
    ref = dy.float() * (y.float() > 0) if y is not None else dy.float()
    for _ in range(3):
        dyb, db = dy_prep(dy, y)
        assert torch.equal(dyb, ref.to(torch.bfloat16))
        assert _rel(db, ref.double().sum(0)) < 1e-5
    sink = torch.randn(N, device=gpu, generator=g)
    want = sink.double() + ref.double().sum(0)
    dyb, db = dy_prep(dy, y, want_bf16=False, db_into=sink)
    assert dyb is None and db is None
    assert _rel(sink, want) < 1e-5
    db1 = dy_prep(dy, y)[1]
    assert torch.equal(db1, dy_prep(dy, y)[1])  # fixed summation order: bitwise reproducible


@pytest.mark.parametrize("mu,wd", [(0.0, 0.0), (0.9, 1e-4)])
def test_sgd(gpu, mu, wd):
    from distributeddataparallel_cifar10_amd.ops import sgd_step_
    g = torch.Generator(device=gpu).manual_seed(11)
    p0 = torch.randn(10001, device=gpu, generator=g)
    ref = p0.clone().requires_grad_()
    opt = torch.optim.SGD([ref], lr=0.05, momentum=mu, weight_decay=wd)
    p = p0.clone()
    buf = torch.zeros_like(p) if mu else None
    first = torch.ones(1, dtype=torch.int32, device=gpu)
    for _ in range(3):
        grad = torch.randn(10001, device=gpu, generator=g)
        ref.grad = grad.clone()
        opt.step()
        sgd_step_(p, grad, 0.05, mu, wd, buf=buf, first=first)
    assert _rel(p, ref.detach()) < 1e-6


@pytest.mark.parametrize("fp8", [False, True])
def test_ops_resnet_step(gpu, fp8):
    """A ResNet-50-structured net (reduced depth for test time) trains one step on the ops path.  Loss and every
    parameter gradient are compared with stock PyTorch fp32; the tolerance is set by stock PyTorch's own bf16
    autocast error on the same step (the ops path must be within 2x of it, +0.02; fp8 forward: 3x, +0.05)."""
    import copy
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    torch.manual_seed(0)
    net = ResNet([1, 1, 1, 1], num_classes=10, zero_init_residual=False).to(gpu)
    ref = copy.deepcopy(net)
    amp = copy.deepcopy(net)
    x = torch.randn(8, 3, 128, 128, device=gpu)
    y = torch.randint(0, 10, (8,), device=gpu)
    loss = cross_entropy(OpsModel(net, fp8=fp8)(x), y)
    loss.backward()
    lref = TF.cross_entropy(ref(x), y)
    lref.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lamp = TF.cross_entropy(amp(x), y)
    lamp.backward()
    k, c = (3.0, 0.12) if fp8 else (2.0, 0.02)
    assert abs(loss.item() - lref.item()) <= k * abs(lamp.item() - lref.item()) + c * max(1.0, lref.item())
    rows = []
    for (n, p), (_, q), (_, r) in zip(net.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        assert p.grad is not None, n
        rows.append((n, _rel(p.grad, q.grad), _rel(r.grad, q.grad)))
    print("\n".join(f"{n:40s} ops {e:.4f}  autocast {a:.4f}" for n, e, a in rows))
    # fp8 forward noise is amplified through the (chaotic, random-init) backward: compare fp8 only near the head,
    # where the gradient is still a function of the forward it perturbs; bf16 is compared everywhere.
    checked = rows if not fp8 else [r for r in rows if r[0].startswith(("fc.", "layer4.0.bn3", "layer4.0.downsample.1"))]
    bad = [(n, e, a) for n, e, a in checked if e > k * a + c]
    assert not bad, bad


@pytest.mark.parametrize("M,N,K", [(20000, 256, 64), (16384, 128, 128), (777, 256, 64), (20000, 256, 256)])
def test_gemm_masked_accumulation_source(gpu, M, N, K):
    """C = A B^T + src * mask bits: in the stream GEMM's epilogue (K <= 128, M >= 16384) or through the masked
    copy before the other kernels (small M, K = 256); against fp32 PyTorch."""
    from distributeddataparallel_cifar10_amd.ops.functional import gemm
    g = torch.Generator(device=gpu).manual_seed(M + K)
    a = _bf(torch.randn(M, K, device=gpu, generator=g))
    b = _bf(torch.randn(N, K, device=gpu, generator=g))
    src = _bf(torch.randn(M, N, device=gpu, generator=g))
    mask = torch.randint(0, 256, (M * N // 8,), device=gpu, generator=g, dtype=torch.int32).to(torch.uint8)
    bits = ((mask.view(-1, 1).int() >> torch.arange(8, device=gpu)) & 1).view(M, N).float()
    out = gemm(a, b, out_dtype=torch.bfloat16, beta=1.0, beta_src=src, beta_mask=mask)
    ref = a.float() @ b.float().t() + src.float() * bits
    assert _rel(out.float(), ref) < 1e-2
    assert torch.equal(src, src.clone())  # the source is read, never written


@pytest.mark.parametrize("layers,batch,img", [([2, 1, 1, 1], 8, 192),   # layer 1: 8 x 48 x 48 = 18432 pixels
                                             ([1, 1, 2, 1], 16, 512)])  # layer 3: 16 x 32 x 32 = 16384 pixels
def test_ops_resnet_masked_identity_gradient_bitwise(gpu, monkeypatch, layers, batch, img):
    """Identity blocks whose conv1 dgrad runs on the stream GEMM take the residual gradient dout * mask in that
    GEMM's epilogue instead of bn3's backward writing it, and downsample blocks hand it to the downsample BN's
    backward as (dout, mask) (ResidualLink): every gradient is bitwise the one of the written path (the masked
    value is exact in bf16 either way; the BN backward kernels use explicit FMAs, so every mode rounds alike)."""
    import copy
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.ops import models as M_
    torch.manual_seed(0)
    net = ResNet(layers, num_classes=10, zero_init_residual=False).to(gpu)
    other = copy.deepcopy(net)
    # the identity block's conv1 dgrad must be stream-GEMM eligible (>= 16384 pixels); the second config puts it in
    # layer 3 (K = 256 there: the masked epilogue source at its largest K)
    x = torch.randn(batch, 3, img, img, device=gpu)
    y = torch.randint(0, 10, (batch,), device=gpu)
    from distributeddataparallel_cifar10_amd.ops import functional as F
    # (the on-the-fly downsample BN changes the forward's residual rounding: off in both, as in the written path)
    monkeypatch.setattr(F, "RES_BN_ON_THE_FLY", False)
    grads = []
    for m, on in ((net, True), (other, False)):
        monkeypatch.setattr(M_, "_MASKED_JOIN", on)
        cross_entropy(OpsModel(m)(x), y).backward()
        grads.append([p.grad.clone() for p in m.parameters()])
    for (n, _), g1, g2 in zip(net.named_parameters(), *grads):
        assert torch.equal(g1, g2), n


def test_downsample_bn_on_the_fly(gpu, monkeypatch):
    """The downsample branch's BN applied inside bn3's apply pass (ResidualLink.lazy: the branch never writes its
    BN output) against the written form: logits, BN running statistics and every parameter gradient agree to bf16
    rounding of the residual, and both against stock fp32 PyTorch."""
    import copy
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(3)
    net = ResNet([2, 1, 1, 1], num_classes=10, zero_init_residual=False).to(gpu)
    other, ref = copy.deepcopy(net), copy.deepcopy(net)
    x = torch.randn(8, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (8,), device=gpu)
    outs, grads = [], []
    for m, on in ((net, True), (other, False)):
        monkeypatch.setattr(F, "RES_BN_ON_THE_FLY", on)
        out = OpsModel(m)(x)
        cross_entropy(out, y).backward()
        outs.append(out.detach())
        grads.append([p.grad.clone() for p in m.parameters()])
    # (random-init residual blocks amplify the residual's bf16 rounding difference through the net: a few %)
    assert _rel(outs[0], outs[1]) < 5e-2
    for b1, b2 in zip(net.buffers(), other.buffers()):
        if b1.dtype.is_floating_point:
            assert _rel(b1, b2) < 1e-2
    lo = ref(x)
    torch.nn.functional.cross_entropy(lo, y).backward()
    # against fp32: as close as the written form
    assert _rel(outs[0], lo.detach()) < 1.5 * _rel(outs[1], lo.detach()) + 1e-3
    for (n, p), q, o in zip(net.named_parameters(), ref.parameters(), other.parameters()):
        assert _rel(p.grad, q.grad) < 1.5 * _rel(o.grad, q.grad) + 2e-3, n


@pytest.mark.parametrize("kind", ["resnet", "netresdeep"])
def test_ops_eval_inference(gpu, kind):
    """Eval-mode forward (inference: BN normalised with the running statistics, k_bn_eval_stats + k_bn_apply)
    on the ops path vs stock fp32 PyTorch in eval mode, with non-trivial running statistics; running buffers
    and num_batches_tracked untouched; the eval path refuses to run under autograd."""
    import copy
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel
    torch.manual_seed(0)
    net = (ResNet([1, 1, 1, 1], num_classes=10, zero_init_residual=False) if kind == "resnet" else NetResDeep()).to(gpu)
    for mod in net.modules():
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_mean.uniform_(-0.2, 0.2)
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.data.uniform_(0.5, 1.5)
            mod.bias.data.uniform_(-0.2, 0.2)
    ref = copy.deepcopy(net).eval()
    ops = OpsModel(net).eval()
    x = torch.randn(8, 3, 96 if kind == "resnet" else 32, 96 if kind == "resnet" else 32, device=gpu)
    bufs = [b.clone() for b in net.buffers()]
    with torch.no_grad():
        y, yref = ops(x), ref(x)
    assert y.dtype == torch.float32 and y.shape == yref.shape
    assert _rel(y, yref) < 3e-2, _rel(y, yref)
    assert all(torch.equal(a, b) for a, b in zip(bufs, net.buffers()))
    with pytest.raises(RuntimeError, match="no_grad"):
        ops(x)


@pytest.mark.parametrize("fp8", [False, True])
def test_ops_resnet_trains(gpu, fp8):
    """20 SGD steps on one fixed batch through the ops path (FlatBucketDDP + HIP SGD with momentum) fit it."""
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD
    torch.manual_seed(1)
    net = OpsModel(ResNet([1, 1, 1, 1], num_classes=10).to(gpu), fp8=fp8)
    ddp = FlatBucketDDP(net)
    opt = FlatSGD(ddp, lr=0.05, momentum=0.9)
    x = torch.randn(16, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (16,), device=gpu)
    losses = []
    for _ in range(20):
        loss = cross_entropy(ddp(x), y)
        opt.zero_grad()
        loss.backward()
        opt.step()
        losses.append(loss.item())
    assert all(torch.isfinite(torch.tensor(losses)))
    assert losses[-1] < 0.5 * losses[0], losses


def test_ops_netresdeep_step(gpu):
    """NetResDeep (reference model/resnet.py) on the ops path: loss and all 9 gradients vs stock fp32 PyTorch,
    within 2x stock bf16 autocast's own error (+0.02); BN running stats updated 10x per forward."""
    import copy
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    torch.manual_seed(0)
    net = NetResDeep().to(gpu)
    ref, amp = copy.deepcopy(net), copy.deepcopy(net)
    x = torch.randn(32, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (32,), device=gpu)
    loss = cross_entropy(OpsModel(net)(x), y)
    loss.backward()
    lref = TF.cross_entropy(ref(x), y)
    lref.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        lamp = TF.cross_entropy(amp(x), y)
    lamp.backward()
    assert abs(loss.item() - lref.item()) <= 2 * abs(lamp.item() - lref.item()) + 0.02
    for (n, p), (_, q), (_, r) in zip(net.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        e, a = _rel(p.grad, q.grad), _rel(r.grad, q.grad)
        assert e <= 2 * a + 0.02, (n, e, a)
    bn, rbn = net.resblocks[0].batch_norm, ref.resblocks[0].batch_norm
    assert int(bn.num_batches_tracked) == int(rbn.num_batches_tracked) == 10
    assert _rel(bn.running_mean, rbn.running_mean) < 2e-2 and _rel(bn.running_var, rbn.running_var) < 2e-2


def test_main_no_ddp_ops_engine(gpu, tmp_path):
    """main_no_ddp.py --engine ops trains NetResDeep on the HIP layer kernels (reference output lines)."""
    import subprocess
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "main_no_ddp.py", "--synthetic", "512", "--epochs", "1", "--engine", "ops"],
                       cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Training loss" in r.stdout and "training time:" in r.stdout


@pytest.mark.parametrize("k,s,p,res_mode,fp8", [(3, 1, 1, 1, False), (1, 1, 0, 2, False), (3, 2, 1, 0, False),
                                                (1, 1, 0, 2, True)])
def test_conv_bn_act(gpu, k, s, p, res_mode, fp8):
    """conv -> BN (stats from the GEMM epilogue) -> ReLU (+ residual) vs torch fp32, forward and backward."""
    from distributeddataparallel_cifar10_amd.ops import conv_bn_act
    g = torch.Generator(device=gpu).manual_seed(k * 10 + res_mode)
    n, h, ci, co = 4, 12, 32, 64 if res_mode != 1 else 32
    conv = torch.nn.Conv2d(ci, co, k, stride=s, padding=p, bias=False).to(gpu)
    bn = torch.nn.BatchNorm2d(co).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
        bn.running_mean.uniform_(-0.1, 0.1)
    rconv, rbn = torch.nn.Conv2d(ci, co, k, stride=s, padding=p, bias=False).to(gpu), torch.nn.BatchNorm2d(co).to(gpu)
    rconv.load_state_dict(conv.state_dict())
    rbn.load_state_dict(bn.state_dict())
    x = _bf(torch.randn(n, h, h, ci, device=gpu, generator=g)).requires_grad_()
    ho = (h + 2 * p - k) // s + 1
    r = _bf(torch.randn(n, ho, ho, co, device=gpu, generator=g)).requires_grad_() if res_mode else None
    y = conv_bn_act(x, conv, bn, r=r, relu=True, fp8=fp8, res_mode=res_mode)
    dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    rr = r.detach().float().permute(0, 3, 1, 2).requires_grad_() if res_mode else None
    with torch.no_grad():
        rconv.weight.copy_(_bf(rconv.weight).float())
    z = rbn(rconv(xr))
    z = torch.relu(z + rr) if res_mode == 2 else torch.relu(z)
    if res_mode == 1:
        z = z + rr
    z.backward(dy.float().permute(0, 3, 1, 2))
    tol = 0.08 if fp8 else 2e-2
    gtol = 0.2 if fp8 else 3e-2  # fp8 forward flips some ReLU masks: the backward inherits that
    assert _rel(y.float().permute(0, 3, 1, 2), z) < tol
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < gtol
    assert _rel(conv.weight.grad, rconv.weight.grad) < gtol
    assert _rel(bn.weight.grad, rbn.weight.grad) < gtol
    assert _rel(bn.running_mean, rbn.running_mean) < 1e-2 and _rel(bn.running_var, rbn.running_var) < 1e-2
    if res_mode:
        assert _rel(r.grad.float().permute(0, 3, 1, 2), rr.grad) < gtol


def test_weight_pack(gpu):
    """WeightPack (one launch for all layers) == the per-layer torch formulation of every GEMM operand: bf16
    forward matrix (3-channel stem zero-padded to 8 channels), flipped dgrad matrix, fp8 copy + amax."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(3)
    convs = [torch.nn.Conv2d(3, 16, 7, stride=2, padding=3, bias=False), torch.nn.Conv2d(32, 64, 3, padding=1),
             torch.nn.Conv2d(128, 64, 1, bias=False)]
    convs = [c.to(gpu) for c in convs]
    pack = F.WeightPack(convs, [convs[2]])
    pack.pack()
    w0 = convs[0].weight.detach()
    ref0 = TF.pad(w0.permute(0, 2, 3, 1), (0, 5)).reshape(16, -1).to(torch.bfloat16)
    assert torch.equal(pack.get(convs[0])["fwd"], ref0)
    assert pack.get(convs[0])["dgrad"] is None
    w1 = convs[1].weight.detach()
    e1 = pack.get(convs[1])
    assert torch.equal(e1["fwd"], F._weight_matrix(w1, 288))
    assert torch.equal(e1["dgrad"], w1.flip(2, 3).permute(1, 2, 3, 0).reshape(32, -1).to(torch.bfloat16))
    e2 = pack.get(convs[2])
    q, amax = F.quantize_fp8(convs[2].weight.detach().reshape(64, 128).contiguous())
    assert torch.equal(e2["amax"], amax) and torch.equal(e2["q8"], q)
    assert torch.equal(e2["dgrad"], convs[2].weight.detach().reshape(64, 128).t().to(torch.bfloat16))
    with torch.no_grad():  # weights change -> the next pack() reflects them (same descriptors)
        convs[1].weight.mul_(-2.0)
    pack.pack()
    assert torch.equal(e1["fwd"], F._weight_matrix(convs[1].weight.detach(), 288))
    # partial 32 x 32 transpose tiles in both dimensions (Cout = 40, Cin * taps = 216)
    conv3 = torch.nn.Conv2d(24, 40, 3, padding=1, bias=False).to(gpu)
    pack3 = F.WeightPack([conv3])
    pack3.pack()
    w3 = conv3.weight.detach()
    assert torch.equal(pack3.get(conv3)["dgrad"], w3.flip(2, 3).permute(1, 2, 3, 0).reshape(24, -1).to(torch.bfloat16))


def test_weight_grad_layout_remap(gpu):
    """Weight gradients written by the GEMM reduce pass straight into [Cout, Cin, KH, KW] (accumulating with
    beta = 1), for the implicit and the explicit (im2col) form."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(5)
    x = _bf(torch.randn(2, 9, 9, 16, device=gpu, generator=g))
    w = torch.randn(24, 16, 3, 3, device=gpu, generator=g)
    geo = F._geom(x, w, 1, 1)
    M = 2 * 9 * 9
    dy = _bf(torch.randn(M, 24, device=gpu, generator=g))
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), w.shape,
                                      dy.float().view(2, 9, 9, 24).permute(0, 3, 1, 2), padding=1)
    out = torch.ones_like(w)
    F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(24, geo.K, M), splits=2, out=out, beta=1.0, wperm=(16, 16, 9))
    assert _rel(out - 1.0, ref) < 1e-5
    cols = torch.empty(M, geo.Kp, dtype=torch.bfloat16, device=gpu)
    from distributeddataparallel_cifar10_amd.ops import _native as N
    N.check(N.lib().dca_ops_im2col(N.ptr(x), N.ptr(cols), geo, N.stream(gpu)), "im2col")
    out2 = torch.empty_like(w)
    F.gemm(dy, cols, ta=True, tb=True, splits=1, out=out2, wperm=(16, 16, 9))
    assert _rel(out2, ref) < 1e-5


@pytest.mark.parametrize("fp8", [False, True])
def test_direct_grads_match_autograd(gpu, fp8):
    """With FlatBucketDDP the ResNet conv / BN gradients are written straight into the flat buffer (grad
    sinks); they must equal the autograd-accumulated gradients of the same step without the wrapper."""
    import copy
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP
    torch.manual_seed(2)
    a = ResNet([1, 1, 1, 1], num_classes=10).to(gpu)
    b = copy.deepcopy(a)
    x = torch.randn(4, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (4,), device=gpu)
    ddp = FlatBucketDDP(OpsModel(a, fp8=fp8))
    ddp.zero_grad()
    cross_entropy(ddp(x), y).backward()
    cross_entropy(OpsModel(b, fp8=fp8)(x), y).backward()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert p.grad is not None and q.grad is not None, n
        assert _rel(p.grad, q.grad) < 1e-6, (n, _rel(p.grad, q.grad))


@pytest.mark.parametrize("M,N,K,splits", [(64, 64, 5000, 7), (64, 200, 3000, 3), (200, 64, 777, 1), (256, 392, 4096, 16),
                                          (136, 1000, 130, 2), (8, 8, 64, 1)])
def test_wgrad_transposed_read_kernel(gpu, M, N, K, splits):
    """Weight-gradient GEMM C = A^T B with both operands pixel-major (k_wgrad: LDS tiles as loaded, MFMA fragments
    by ds_read_b64_tr_b16) for every tile shape (64/128 x 64/128), ragged M, N, K and split-K, vs fp32 torch."""
    from distributeddataparallel_cifar10_amd.ops import gemm
    g = torch.Generator(device=gpu).manual_seed(M + N + K)
    a = _bf(torch.randn(K, M, device=gpu, generator=g))
    b = _bf(torch.randn(K, N, device=gpu, generator=g) * torch.linspace(0.5, 2.0, N, device=gpu))
    ref = a.float().t() @ b.float()
    out = gemm(a, b, ta=True, tb=True, splits=splits)
    assert _rel(out, ref) < 1e-5, _rel(out, ref)


@pytest.mark.parametrize("M,N,K,splits", [(256, 256, 4096, 4), (512, 384, 3000, 7), (264, 136, 777, 1),
                                          (1024, 256, 50176, 64), (256, 1160, 200, 1), (256, 64, 4096, 4),
                                          (64, 576, 5000, 8), (128, 1152, 3000, 5), (64, 264, 777, 1),
                                          (120, 512, 640, 2)])
def test_wgrad_pingpong_kernel(gpu, M, N, K, splits):
    """Weight gradients on k_wgrad_pp (the larger of M / N along the 256-row side, the smaller as a 256 / 128 / 64
    column tile; LDS-DMA with swizzled source chunks, transposed fragment reads, two ping-pong wave groups):
    ragged M, N, K tails, split-K and the swapped (M < 256) form, vs fp32 torch."""
    from distributeddataparallel_cifar10_amd.ops import gemm
    g = torch.Generator(device=gpu).manual_seed(M * 7 + N + K)
    a = _bf(torch.randn(K, M, device=gpu, generator=g))
    b = _bf(torch.randn(K, N, device=gpu, generator=g) * torch.linspace(0.5, 2.0, N, device=gpu))
    ref = a.float().t() @ b.float()
    out = gemm(a, b, ta=True, tb=True, splits=splits)
    assert _rel(out, ref) < 1e-5, _rel(out, ref)


@pytest.mark.parametrize("n,h,c,co,k,s,p", [(3, 13, 64, 256, 3, 1, 1), (2, 14, 128, 512, 3, 2, 1),
                                            (2, 12, 256, 264, 1, 2, 0), (4, 7, 512, 256, 3, 1, 1),
                                            (3, 14, 64, 64, 3, 1, 1), (2, 15, 128, 128, 3, 2, 1),
                                            (2, 20, 8, 64, 7, 2, 3)])
def test_wgrad_pingpong_implicit_conv(gpu, n, h, c, co, k, s, p):
    """Implicit-im2col weight gradients (conv = 2) on k_wgrad_pp, as its column side (Cout >= 256) or its row side
    (swapped: Cout 64 / 128, incl. the 8-channel 7x7/2 stem): taps straddling tiles, zero padding, stride 2, ragged
    pixel counts, written into torch's [Cout, Cin, KH, KW] layout."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(n * h + c + co)
    x = _bf(torch.randn(n, h, h, c, device=gpu, generator=g))
    w = torch.empty(co, c, k, k, device=gpu)
    geo = F._geom(x, w, s, p)
    M = n * geo.Ho * geo.Wo
    dy = _bf(torch.randn(M, co, device=gpu, generator=g))
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), w.shape,
                                      dy.float().view(n, geo.Ho, geo.Wo, co).permute(0, 3, 1, 2), stride=s, padding=p)
    out = torch.empty_like(w)
    F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(co, geo.K, M), splits=F._wgrad_splits(co, geo.K, M), out=out,
           wperm=(c, c, k * k))
    assert _rel(out, ref) < 1e-5, _rel(out, ref)


@pytest.mark.parametrize("n,h,w,c", [(2, 9, 11, 64), (4, 56, 56, 64), (3, 17, 5, 64), (2, 7, 64, 64), (2, 5, 40, 64),
                                     (1, 6, 70, 64), (4, 28, 28, 128), (3, 9, 11, 128), (2, 5, 32, 128),
                                     (1, 6, 40, 128)])
def test_wgrad3x3_rows(gpu, n, h, w, c):
    """The 64- / 128-channel 3x3 / pad 1 weight gradients as the model calls them (implicit split count): W <= 64 /
    32 run the row-ring k_wgrad3x3_rows<ceil(W / 32), C> (one and two 32-pixel chunks, pixels past W, padding rows,
    one split slab per workgroup -- per output-channel half for 128), W = 70 / 40 the k_wgrad / ping-pong fallbacks;
    against torch fp32 in torch's [Cout, Cin, 3, 3] layout."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(n * h + w + c)
    x = _bf(torch.randn(n, h, w, c, device=gpu, generator=g))
    wt = torch.empty(c, c, 3, 3, device=gpu)
    geo = F._geom(x, wt, 1, 1)
    M = n * geo.Ho * geo.Wo
    dy = _bf(torch.randn(M, c, device=gpu, generator=g))
    ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), wt.shape,
                                      dy.float().view(n, geo.Ho, geo.Wo, c).permute(0, 3, 1, 2), stride=1, padding=1)
    out = torch.full_like(wt, float("nan"))
    F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(c, geo.K, M), splits=F._wgrad_splits(c, geo.K, M, True, row_w=w),
           out=out, wperm=(c, c, 9))
    assert _rel(out, ref) < 1e-5, _rel(out, ref)


def test_wgrad_pingpong_forms(gpu):
    """Every weight-gradient form the dispatch routes to k_wgrad_pp -- 256 x 256 and 256 x 128 column tiles, the
    swapped plain form (64 < M <= 128), the implicit-im2col B operand -- and the k_wgrad fallbacks beside them
    (M = 64, the 7x7 stem), with ragged tails, against torch fp32.  (The 64-wide and swapped-implicit ping-pong
    forms measured slower and were removed in round 5.)"""
    from distributeddataparallel_cifar10_amd import ops
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(0)
    bf = torch.bfloat16
    for M, N, K, sp in [(256, 256, 4096, 4), (512, 128, 3000, 5), (128, 512, 2999, 3), (64, 264, 777, 1),
                        (264, 72, 999, 3)]:
        a = torch.randn(K, M, device=gpu, generator=g).to(bf)
        b = (torch.randn(K, N, device=gpu, generator=g) * torch.linspace(0.5, 2.0, N, device=gpu)).to(bf)
        assert _rel(ops.gemm(a, b, ta=True, tb=True, splits=sp), a.float().t() @ b.float()) < 1e-5, (M, N, K)
    for n, h, c, co, k, s, p in [(3, 14, 64, 256, 3, 1, 1), (2, 15, 128, 128, 3, 2, 1), (2, 20, 8, 64, 7, 2, 3),
                                 (2, 13, 64, 256, 1, 1, 0)]:
        x = torch.randn(n, h, h, c, device=gpu, generator=g).to(bf)
        w = torch.empty(co, c, k, k, device=gpu)
        geo = F._geom(x, w, s, p)
        M = n * geo.Ho * geo.Wo
        dy = torch.randn(M, co, device=gpu, generator=g).to(bf)
        ref = torch.nn.grad.conv2d_weight(x.float().permute(0, 3, 1, 2), w.shape,
                                          dy.float().view(n, geo.Ho, geo.Wo, co).permute(0, 3, 1, 2), stride=s,
                                          padding=p)
        o = torch.empty_like(w)
        F.gemm(dy, x, ta=True, conv=2, geom=geo, mnk=(co, geo.K, M), splits=F._wgrad_splits(co, geo.K, M), out=o,
               wperm=(c, c, k * k))
        assert _rel(o, ref) < 1e-5, (n, h, c, co, k)


def test_main_no_ddp_resnet50_auto_ops(gpu):
    """--model resnet50 on a GPU resolves to the ops engine (HIP kernels, packed weights, gradient sinks)."""
    import subprocess
    import sys
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, "main_no_ddp.py", "--synthetic", "256", "--epochs", "1", "--max-steps", "3",
                        "--model", "resnet50"], cwd=root, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Training loss" in r.stdout and "training time:" in r.stdout


def test_ops_resnet_overlapped_sgd_matches(gpu):
    """FlatSGD(overlap=True) on the GPU (bucket updates on the side stream during the backward, momentum) gives
    the same parameters as the post-backward flat SGD, step for step."""
    import copy
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD
    torch.manual_seed(4)
    a = ResNet([1, 1, 1, 1], num_classes=10).to(gpu)
    b = copy.deepcopy(a)
    da = FlatBucketDDP(OpsModel(a), bucket_cap_mb=1.0, first_bucket_mb=0.2)
    db = FlatBucketDDP(OpsModel(b), bucket_cap_mb=1.0, first_bucket_mb=0.2)
    oa = FlatSGD(da, lr=0.05, momentum=0.9, weight_decay=1e-4)
    ob = FlatSGD(db, lr=0.05, momentum=0.9, weight_decay=1e-4, overlap=True)
    x = torch.randn(4, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (4,), device=gpu)
    for step in range(3):
        for d, o in ((da, oa), (db, ob)):
            o.zero_grad()
            cross_entropy(d(x), y).backward()
            o.step()
        torch.cuda.synchronize()
        assert sorted(db.bucket_fire_order) == list(range(len(db.buckets)))
        assert torch.equal(da.flat, db.flat), (step, _rel(db.flat, da.flat))


@pytest.mark.parametrize("s", [1, 2])
def test_conv_bn_act_fp8_implicit_3x3(gpu, s):
    """fp8 forward of a 3x3 conv as an implicit GEMM over the input's fp8 copy (packed fp8 weights), with BN in
    the epilogue, vs torch fp32: forward within fp8 tolerance, backward (bf16) unaffected in structure."""
    from distributeddataparallel_cifar10_amd.ops import conv_bn_act
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(11 + s)
    n, h, ci, co = 4, 14, 64, 32
    conv = torch.nn.Conv2d(ci, co, 3, stride=s, padding=1, bias=False).to(gpu)
    bn = torch.nn.BatchNorm2d(co).to(gpu)
    rconv, rbn = torch.nn.Conv2d(ci, co, 3, stride=s, padding=1, bias=False).to(gpu), torch.nn.BatchNorm2d(co).to(gpu)
    rconv.load_state_dict(conv.state_dict())
    rbn.load_state_dict(bn.state_dict())
    pack = F.WeightPack([conv], [conv])
    pack.pack()
    x = _bf(torch.randn(n, h, h, ci, device=gpu, generator=g)).requires_grad_()
    y = conv_bn_act(x, conv, bn, relu=True, fp8=True, packed=pack.get(conv))
    dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    z = torch.relu(rbn(rconv(xr)))
    z.backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(y.float().permute(0, 3, 1, 2), z) < 0.08
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 0.2
    assert _rel(conv.weight.grad, rconv.weight.grad) < 0.2


def test_nchw_to_nhwc8(gpu):
    from distributeddataparallel_cifar10_amd.ops import functional as F
    x = torch.randn(3, 3, 17, 19, device=gpu)
    y = F.nchw_to_nhwc8(x)
    ref = TF.pad(x.permute(0, 2, 3, 1), (0, 5)).to(torch.bfloat16)
    assert y.shape == (3, 17, 19, 8) and torch.equal(y, ref)


def test_ops_resnet_counts_batches_once_per_forward(gpu):
    """The batched num_batches_tracked increment: every BN counts exactly one batch per forward."""
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    net = ResNet([1, 1, 1, 1], num_classes=10).to(gpu)
    m = OpsModel(net)
    x = torch.randn(2, 3, 64, 64, device=gpu)
    y = torch.randint(0, 10, (2,), device=gpu)
    for _ in range(3):
        cross_entropy(m(x), y).backward()
    counts = {int(b.num_batches_tracked) for b in net.modules() if isinstance(b, torch.nn.BatchNorm2d)}
    assert counts == {3}, counts


@pytest.mark.parametrize("n,h,ci,co", [(6, 64, 64, 64), (3, 30, 64, 128)])
def test_bn_pool_fused_matches_two_pass(gpu, n, h, ci, co):
    """conv -> BN + ReLU + 3x3/2/1 max pool in one pass each way (the ResNet stem, k_bn_pool_*) against the
    two-pass form (k_bn_apply + k_maxpool_fwd_k3s2, k_maxpool_bwd_k3s2 + the BN backward): forward output and argmax
    bitwise, BN running statistics bitwise, gradients to the summation order of the BN backward sums; and both
    against torch fp32."""
    import copy
    from distributeddataparallel_cifar10_amd.ops import conv_bn_act, max_pool2d
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(n * h + co)
    conv = torch.nn.Conv2d(ci, co, 3, padding=1, bias=False).to(gpu)
    bn = torch.nn.BatchNorm2d(co).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5, generator=g)
        bn.bias.uniform_(-0.5, 0.5, generator=g)
    conv2, bn2 = copy.deepcopy(conv), copy.deepcopy(bn)
    x = _bf(torch.randn(n, h, h, ci, device=gpu, generator=g))
    x1, x2 = x.clone().requires_grad_(), x.clone().requires_grad_()
    assert F.bn_pool_ok(x1, conv)
    y1 = conv_bn_act(x1, conv, bn, relu=True, pool=True)
    y2 = max_pool2d(conv_bn_act(x2, conv2, bn2, relu=True), 3, 2, 1)
    assert y1.shape == (n, h // 2, h // 2, co) and torch.equal(y1, y2)
    assert torch.equal(bn.running_mean, bn2.running_mean) and torch.equal(bn.running_var, bn2.running_var)
    dp = _bf(torch.randn(y1.shape, device=gpu, generator=g))
    y1.backward(dp)
    y2.backward(dp)
    assert _rel(bn.weight.grad, bn2.weight.grad) < 1e-5 and _rel(bn.bias.grad, bn2.bias.grad) < 1e-5
    assert _rel(conv.weight.grad, conv2.weight.grad) < 1e-3
    assert _rel(x1.grad.float(), x2.grad.float()) < 1e-2
    # torch fp32 reference of the same module chain
    rc, rb = copy.deepcopy(conv2), torch.nn.BatchNorm2d(co).to(gpu)
    rb.load_state_dict({k: v for k, v in bn.state_dict().items() if k not in ("running_mean", "running_var")},
                       strict=False)
    rc.weight.grad = rb.weight.grad = None
    xr = x.float().permute(0, 3, 1, 2).requires_grad_()
    z = TF.max_pool2d(torch.relu(rb(torch.nn.functional.conv2d(xr, _bf(rc.weight).float(), padding=1))), 3, 2, 1)
    z.backward(dp.float().permute(0, 3, 1, 2))
    assert _rel(y1.float().permute(0, 3, 1, 2), z) < 2e-2
    assert _rel(bn.weight.grad, rb.weight.grad) < 2e-2 and _rel(bn.bias.grad, rb.bias.grad) < 2e-2
    # the input gradient runs through the BN backward's cancellation in bf16 (dz - mean - xhat * mean(dz xhat)):
    # the fused form must be as close to fp32 as the two-pass form
    e1 = _rel(x1.grad.float().permute(0, 3, 1, 2), xr.grad)
    e2 = _rel(x2.grad.float().permute(0, 3, 1, 2), xr.grad)
    assert e1 < 1.05 * e2 + 1e-3 and e1 < 0.15, (e1, e2)


def test_strided_1x1_conv_on_stream_kernel(gpu):
    """A strided 1x1 (downsample) convolution with N % 128 == 0 and M >= 16384 -- the production route onto the
    persistent stream kernel's implicit-conv form -- with the fused BN column statistics, vs torch fp32."""
    from distributeddataparallel_cifar10_amd import ops
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(21)
    n, h, c, co = 24, 56, 128, 384  # M = 24 x 28 x 28 = 18816
    x = _bf(torch.randn(n, h, h, c, device=gpu, generator=g))
    w = torch.randn(co, c, 1, 1, device=gpu, generator=g) * 0.05
    geo = F._geom(x, w, 2, 0)
    M = n * geo.Ho * geo.Wo
    parts = torch.zeros((M + 127) // 128, co, 2, device=gpu)
    shift = torch.randn(co, device=gpu, generator=g) * 0.1
    y = ops.gemm(x, F._weight_matrix(w, geo.K), conv=1, geom=geo, mnk=(M, co, geo.K), out_dtype=torch.bfloat16,
                 col_stats=parts, stats_shift=shift)
    ref = torch.nn.functional.conv2d(x.float().permute(0, 3, 1, 2), _bf(w).float(), stride=2)
    assert _rel(y.float().view(n, geo.Ho, geo.Wo, co).permute(0, 3, 1, 2), ref) < 5e-3
    d = y.float() - shift
    assert _rel(parts[..., 0].sum(0), d.sum(0)) < 1e-4 and _rel(parts[..., 1].sum(0), (d * d).sum(0)) < 1e-4


@pytest.mark.parametrize("k,p", [(3, 1), (1, 0)])
def test_strided_conv_subpixel_input_grad(gpu, k, p):
    """Stride-2 conv input gradient by parity classes (implicit stride-1 convs over dY, GEMM epilogue rows
    remapped into dX) with the packed class matrices, vs torch fp32; and accumulating into a GradJoin buffer."""
    from distributeddataparallel_cifar10_amd.ops import conv_bn_act
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(21 + k)
    n, h, ci, co = 2, 14, 64, 128
    conv = torch.nn.Conv2d(ci, co, k, stride=2, padding=p, bias=False).to(gpu)
    bn = torch.nn.BatchNorm2d(co).to(gpu)
    rconv, rbn = torch.nn.Conv2d(ci, co, k, stride=2, padding=p, bias=False).to(gpu), torch.nn.BatchNorm2d(co).to(gpu)
    rconv.load_state_dict(conv.state_dict())
    rbn.load_state_dict(bn.state_dict())
    pack = F.WeightPack([conv])
    pack.pack()
    e = pack.get(conv)
    assert (e["classes"] is not None) == (k > 1) and (k > 1 or e["dgrad"] is not None)
    x = _bf(torch.randn(n, h, h, ci, device=gpu, generator=g)).requires_grad_()
    y = conv_bn_act(x, conv, bn, relu=True, packed=e)
    dy = _bf(torch.randn(y.shape, device=gpu, generator=g))
    y.backward(dy)
    xr = x.detach().float().permute(0, 3, 1, 2).requires_grad_()
    with torch.no_grad():
        rconv.weight.copy_(_bf(rconv.weight).float())
    torch.relu(rbn(rconv(xr))).backward(dy.float().permute(0, 3, 1, 2))
    assert _rel(x.grad.float().permute(0, 3, 1, 2), xr.grad) < 3e-2
    # accumulate mode: a GradJoin whose buffer already holds another consumer's gradient
    join = F.GradJoin(2)
    seed = _bf(torch.randn(n, h, h, ci, device=gpu, generator=g))
    join.contribute(seed.clone())
    x2 = x.detach().clone().requires_grad_()
    y2 = conv_bn_act(x2, conv, bn, relu=True, packed=e, x_join=join)
    y2.backward(dy)
    assert _rel(x2.grad.float(), seed.float() + x.grad.float()) < 2e-2


@pytest.mark.parametrize("n,h,w,c", [(2, 9, 11, 64), (4, 56, 56, 64), (3, 17, 5, 64), (2, 7, 64, 64), (1, 5, 40, 64),
                                     (2, 3, 20, 64), (1, 6, 70, 64), (4, 28, 28, 128), (3, 9, 11, 128),
                                     (2, 5, 16, 128), (1, 6, 40, 128)])
def test_direct_conv_3x3_64(gpu, n, h, w, c):
    """The 64- and 128-channel 3x3 / pad 1 convolutions (bf16 output + fused BN column statistics) against torch
    fp32 on the same bf16-rounded operands: padding on every border, M tails, the statistics rows (all of them
    written: the buffer starts as NaN).  64 channels: W <= 64 runs the row-ring kernel k_conv3x3_rows<ceil(W / 16)>
    (one to four fragments), W = 70 the per-pixel k_direct_conv<64, 3, 3>; 128 channels: W <= 32 runs
    k_conv3x3_rows<ceil(W / 16), 128> (ResNet-50's layer 2 at 28 x 28), W = 40 the stream GEMM."""
    from distributeddataparallel_cifar10_amd import ops
    from distributeddataparallel_cifar10_amd.ops import functional as F
    g = torch.Generator(device=gpu).manual_seed(n * h + w + c)
    x = torch.randn(n, h, w, c, device=gpu, generator=g).to(torch.bfloat16)
    wt = torch.randn(c, c, 3, 3, device=gpu, generator=g) * (0.05 if c == 64 else 0.035)
    geo = F._geom(x, wt, 1, 1)
    wm = F._weight_matrix(wt, geo.K)
    M = geo.N * geo.Ho * geo.Wo
    shift = torch.randn(c, device=gpu, generator=g) * 0.1
    parts = torch.full(((M + 127) // 128, c, 2), float("nan"), device=gpu)
    y = ops.gemm(x, wm, conv=1, geom=geo, mnk=(M, c, geo.K), out_dtype=torch.bfloat16, col_stats=parts,
                 stats_shift=shift)
    ref = TF.conv2d(x.float().permute(0, 3, 1, 2), wt.to(torch.bfloat16).float(), padding=1)
    ref = ref.permute(0, 2, 3, 1).reshape(M, c)
    assert _rel(y, ref) < 5e-3
    d = y.float() - shift
    assert _rel(parts[..., 0].sum(0), d.sum(0)) < 1e-4 and _rel(parts[..., 1].sum(0), (d * d).sum(0)) < 1e-4
