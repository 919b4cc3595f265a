"""The space-to-depth form of the 7x7/2/3 stem (ops/functional.py stem_s2d_index / nchw_to_s2d16): a 4x4 stride-1
conv over the 16-channel s2d input equals torch's 7x7 / 2 conv, and the 4x4 weight gradient maps back to torch's
[Co, C, 7, 7] gradient (CPU: the index tables in plain torch; GPU: the kernels inside OpsModel)."""
import pytest
import torch
import torch.nn.functional as TF


def _s2d_ref(x):
    """Plain-torch space-to-depth of NCHW x for the 7x7/2/3 stem: [N, Ho + 3, Wo + 3, 16] (ops layout)."""
    from distributeddataparallel_cifar10_amd.ops.functional import S2D_C, S2D_PAD, S2D_TAPS
    n, c, h, w = x.shape
    ho, wo = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    hs, ws = ho + S2D_TAPS - 1, wo + S2D_TAPS - 1
    xp = torch.zeros(n, c, 2 * hs + 2, 2 * ws + 2, dtype=x.dtype)
    xp[:, :, S2D_PAD:S2D_PAD + h, S2D_PAD:S2D_PAD + w] = x
    y = torch.zeros(n, hs, ws, S2D_C, dtype=x.dtype)
    for ph in (0, 1):
        for pw in (0, 1):
            y[..., (2 * ph + pw) * c:(2 * ph + pw + 1) * c] = xp[:, :, ph:ph + 2 * hs:2, pw:pw + 2 * ws:2].permute(0, 2, 3, 1)
    return y


@pytest.mark.parametrize("c,h", [(3, 224), (3, 37), (1, 20), (4, 16)])
def test_stem_s2d_index_cpu(c, h):
    from distributeddataparallel_cifar10_amd.ops.functional import stem_s2d_index
    torch.manual_seed(c + h)
    conv = torch.nn.Conv2d(c, 16, 7, stride=2, padding=3, bias=False).double()
    x = torch.randn(2, c, h, h + 3, dtype=torch.float64)
    fwd, back = stem_s2d_index(conv)
    w = conv.weight.detach()
    wp = torch.where(fwd >= 0, w.reshape(-1)[fwd.clamp_min(0)], torch.zeros((), dtype=w.dtype))
    w4 = wp.view(16, 4, 4, 16).permute(0, 3, 1, 2)  # [Co, 16, 4, 4] (torch layout of the 4x4 conv)
    xs = _s2d_ref(x).permute(0, 3, 1, 2)
    ref = TF.conv2d(x, w, stride=2, padding=3)
    out = TF.conv2d(xs, w4)
    assert out.shape == ref.shape
    assert (out - ref).abs().max().item() < 1e-10
    # weight gradient: the 4x4 conv's gradient, mapped back, equals the 7x7 one
    dy = torch.randn(ref.shape, dtype=torch.float64)
    g7 = torch.nn.grad.conv2d_weight(x, w.shape, dy, stride=2, padding=3)
    g4 = torch.nn.grad.conv2d_weight(xs, w4.shape, dy)
    mapped = g4.reshape(16, -1).index_select(1, back).view(w.shape)
    assert (mapped - g7).abs().max().item() < 1e-9


@pytest.mark.gpu
def test_stem_s2d_conv_kernels_match_torch(gpu):
    """The stem conv alone on the GPU kernels: s2d operand (k_nchw_to_s2d16), the gathered 4x4 weight matrix
    (WeightPack, k_pack_gather), the 4x4 implicit GEMM forward, and the 4x4 implicit weight-gradient GEMM mapped back
    to [Co, 3, 7, 7], against torch fp32 on the same bf16-rounded operands."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(1)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(gpu)
    pack = F.WeightPack([conv], (), [conv])
    pack.pack()
    e = pack.get(conv)
    x = torch.randn(3, 3, 50, 46, device=gpu)
    xs = F.nchw_to_s2d16(x)
    assert torch.equal(xs.cpu().float(), _s2d_ref(x.cpu().to(torch.bfloat16).float()))
    wg, st, pd = F._s2d_args(conv.weight, 2, 3, e)
    g = F._geom(xs, wg, st, pd)
    M = g.N * g.Ho * g.Wo
    y = F.gemm(xs, e["fwd"], conv=1, geom=g, mnk=(M, 64, g.K), out_dtype=torch.float32)
    xr = x.to(torch.bfloat16).float()
    wr = conv.weight.detach().to(torch.bfloat16).float()
    ref = TF.conv2d(xr, wr, stride=2, padding=3)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    assert rel(y.view(g.N, g.Ho, g.Wo, 64).permute(0, 3, 1, 2), ref) < 1e-5
    dy = torch.randn(M, 64, device=gpu).to(torch.bfloat16)
    d4 = torch.empty(64, 16, 4, 4, device=gpu)
    F.gemm(dy, xs, ta=True, conv=2, geom=g, mnk=(64, g.K, M), splits=F._wgrad_splits(64, g.K, M), out=d4,
           wperm=(16, 16, 16))
    dw = d4.view(64, -1).index_select(1, e["s2d"]["back_idx"]).view(64, 3, 7, 7)
    gref = torch.nn.grad.conv2d_weight(xr, wr.shape, dy.float().view(g.N, g.Ho, g.Wo, 64).permute(0, 3, 1, 2),
                                       stride=2, padding=3)
    assert rel(dw, gref) < 1e-5


@pytest.mark.gpu
def test_stem_s2d_ops_model_stem(gpu):
    """OpsModel's space-to-depth stem end to end (s2d kernel, 4x4 conv, BN, ReLU, max pool) against torch fp32; its
    conv1 weight gradient against torch's on the same upstream gradient (bf16 ties in the max pool route a few
    gradients to other pixels, so the gradient is compared by direction)."""
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(0)
    m = ResNet([1, 1, 1, 1], num_classes=10).to(gpu)
    ops = OpsModel(m)
    x = torch.randn(4, 3, 64, 72, device=gpu)
    h = ops.begin(x)
    assert ops._s2d is m.conv1 and h.shape[-1] == F.S2D_C
    out = ops.stem(h, m.conv1, m.bn1)
    dy = torch.randn(out.shape, device=gpu)
    out.float().backward(dy.to(torch.bfloat16).float())
    wr = m.conv1.weight.detach().to(torch.bfloat16).float().requires_grad_()
    xr = x.to(torch.bfloat16).float()
    yr = TF.conv2d(xr, wr, stride=2, padding=3)
    zr = TF.max_pool2d(TF.relu(TF.batch_norm(yr, None, None, m.bn1.weight.detach(), m.bn1.bias.detach(),
                                             training=True)), 3, 2, 1)
    zr.backward(dy.to(torch.bfloat16).float().permute(0, 3, 1, 2))
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    assert rel(out.float().permute(0, 3, 1, 2), zr) < 2e-2
    cos = TF.cosine_similarity(m.conv1.weight.grad.flatten().double(), wr.grad.flatten().double(), dim=0).item()
    assert cos > 0.99, cos


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(3, 50, 46), (2, 224, 224), (5, 37, 64), (1, 40, 250), (1, 30, 262)])
def test_stem_conv_kernel_bf16_stats(gpu, n, h, w):
    """The dedicated s2d stem kernels (bf16 output with the fused BN column statistics, the form the ops model's stem
    calls: k_conv_s2d_rows up to 128 s2d pixels per row -- w = 250 is the 8-fragment edge -- and k_direct_conv<16, 4,
    4> beyond, w = 262) against torch fp32 on the same bf16-rounded operands: output, and the statistics rows (all of
    them written: the buffer starts as NaN)."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(n + h)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(gpu)
    pack = F.WeightPack([conv], (), [conv])
    pack.pack()
    e = pack.get(conv)
    x = torch.randn(n, 3, h, w, device=gpu)
    xs = F.nchw_to_s2d16(x)
    wg, st, pd = F._s2d_args(conv.weight, 2, 3, e)
    g = F._geom(xs, wg, st, pd)
    M = g.N * g.Ho * g.Wo
    shift = torch.randn(64, device=gpu) * 0.1
    parts = torch.full(((M + 127) // 128, 64, 2), float("nan"), device=gpu)
    y = F.gemm(xs, e["fwd"], conv=1, geom=g, mnk=(M, 64, g.K), out_dtype=torch.bfloat16, col_stats=parts,
               stats_shift=shift)
    xr = x.to(torch.bfloat16).float()
    wr = conv.weight.detach().to(torch.bfloat16).float()
    ref = TF.conv2d(xr, wr, stride=2, padding=3).permute(0, 2, 3, 1).reshape(M, 64)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    assert rel(y.float(), ref) < 5e-3
    d = y.float() - shift
    assert rel(parts[..., 0].sum(0), d.sum(0)) < 1e-4 and rel(parts[..., 1].sum(0), (d * d).sum(0)) < 1e-4


@pytest.mark.gpu
@pytest.mark.parametrize("n,h,w", [(3, 50, 46), (2, 224, 224), (1, 40, 250), (1, 30, 262)])
def test_stem_wgrad_rows(gpu, n, h, w):
    """The s2d stem's weight gradient as the ops model calls it (implicit split count): k_wgrad_s2d_rows up to 128
    s2d pixels per row (one to four 32-pixel chunks, image boundaries inside a workgroup's rows; w = 250 is the
    128-pixel edge) and the k_wgrad fallback beyond (w = 262), mapped back to [Co, 3, 7, 7], against torch fp32."""
    from distributeddataparallel_cifar10_amd.ops import functional as F
    torch.manual_seed(n * h + w)
    conv = torch.nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False).to(gpu)
    pack = F.WeightPack([conv], (), [conv])
    pack.pack()
    e = pack.get(conv)
    x = torch.randn(n, 3, h, w, device=gpu)
    xs = F.nchw_to_s2d16(x)
    wg, st, pd = F._s2d_args(conv.weight, 2, 3, e)
    g = F._geom(xs, wg, st, pd)
    M = g.N * g.Ho * g.Wo
    dy = torch.randn(M, 64, device=gpu).to(torch.bfloat16)
    d4 = torch.full((64, 16, 4, 4), float("nan"), device=gpu)
    F.gemm(dy, xs, ta=True, conv=2, geom=g, mnk=(64, g.K, M), splits=F._wgrad_splits(64, g.K, M, True, row_w=g.W),
           out=d4, wperm=(16, 16, 16))
    dw = d4.view(64, -1).index_select(1, e["s2d"]["back_idx"]).view(64, 3, 7, 7)
    xr = x.to(torch.bfloat16).float()
    gref = torch.nn.grad.conv2d_weight(xr, conv.weight.shape, dy.float().view(g.N, g.Ho, g.Wo, 64).permute(0, 3, 1, 2),
                                       stride=2, padding=3)
    rel = lambda a, b: ((a.double() - b.double()).norm() / b.double().norm()).item()  # noqa: E731
    assert rel(dw, gref) < 1e-5, rel(dw, gref)
