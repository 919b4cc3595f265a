"""Plain-PyTorch fp32 oracle of one NetResDeep training step (the numerical reference for the HIP engine).

Mirrors reference ``main.py:33-41`` + ``model/resnet.py:15-37`` op for op, but unrolls the 10 applications of the
shared ResBlock so every per-application intermediate (block inputs x_i, conv outputs y_i and their gradients)
can be compared with the engine's workspace.  Runs on CPU (or any device) in fp32.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

CIFAR_MEAN = (0.4915, 0.4823, 0.4468)  # reference main.py:56
CIFAR_STD = (0.2470, 0.2435, 0.2616)   # reference main.py:57


def normalize_u8(imgs_u8: torch.Tensor) -> torch.Tensor:
    """uint8 [B,3,32,32] -> ToTensor (/255) -> Normalize, exactly the per-element formula of the kernels."""
    x = imgs_u8.to(torch.float32) / 255.0
    mean = torch.tensor(CIFAR_MEAN, dtype=torch.float32, device=x.device).view(1, 3, 1, 1)
    std = torch.tensor(CIFAR_STD, dtype=torch.float32, device=x.device).view(1, 3, 1, 1)
    return (x - mean) / std


def _bf(t: torch.Tensor) -> torch.Tensor:
    return t.to(torch.bfloat16).to(torch.float32)


class _ConvBF16Operands(torch.autograd.Function):
    """3x3/pad-1 conv whose MFMA operands are rounded to bf16 exactly where the HIP kernels round them:
    forward (x, W), dgrad (dy, W), wgrad (dy, x); products/accumulation in fp32."""

    @staticmethod
    def forward(ctx, x, w, b):
        xr, wr = _bf(x), _bf(w)
        ctx.save_for_backward(xr, wr)
        ctx.has_bias = b is not None
        return F.conv2d(xr, wr, b, padding=1)

    @staticmethod
    def backward(ctx, gy):
        xr, wr = ctx.saved_tensors
        gyr = _bf(gy)
        gx = torch.nn.grad.conv2d_input(xr.shape, wr, gyr, padding=1) if ctx.needs_input_grad[0] else None
        gw = torch.nn.grad.conv2d_weight(xr, wr.shape, gyr, padding=1)
        gb = gy.sum((0, 2, 3)) if ctx.has_bias else None
        return gx, gw, gb


def _conv(mod, x, bf16_operands: bool):
    if bf16_operands:
        return _ConvBF16Operands.apply(x, mod.weight, mod.bias)
    return mod(x)


def _forced(t: torch.Tensor, value) -> torch.Tensor:
    """Straight-through: the forward takes `value`, the gradient flows to `t` unchanged."""
    if value is None:
        return t
    return t + (value.to(t.dtype) - t).detach()


def reference_step(model, imgs_u8: torch.Tensor, labels: torch.Tensor, lr: float = 1e-2, apply_sgd: bool = True,
                   bf16_operands: bool = False, fc1_bf16: bool = False, force: dict | None = None):
    """One SGD step of `model` (mutated in place).  Returns a dict of intermediates and gradients.

    bf16_operands=True emulates the engine's bf16 mode (bf16 MFMA operands, fp32 everything else), so the
    comparison isolates kernel bugs from bf16 rounding; fc1_bf16=True additionally rounds the fc1 weight the
    persistent engine reads (its head keeps a bf16 copy of fc1.weight).

    force={"c1": NCHW conv1 output (pre-ReLU), "x0": NCHW stem output, "y": [10 NCHW conv outputs]} (the
    engine's own forward, any subset): every forced tensor
    enters the graph straight-through, so BatchNorm statistics, ReLU masks and max-pool argmaxes downstream of it
    are the engine's.  The backward then differs from the engine's only by arithmetic, not by the mask flips that
    near-zero pre-activations cause between two independently rounded forwards (flip-aware comparison)."""
    force = force or {}
    x = normalize_u8(imgs_u8)
    blk = model.resblocks[0]
    c1 = _forced(_conv(model.conv1, x, bf16_operands), force.get("c1"))
    out0 = _forced(F.max_pool2d(torch.relu(c1), 2), force.get("x0"))
    xs, ys = [out0], []
    out0.retain_grad()
    cur = out0
    for i in range(len(model.resblocks)):
        y = _forced(_conv(blk.conv, cur, bf16_operands), force["y"][i] if "y" in force else None)
        y.retain_grad()
        ys.append(y)
        nxt = torch.relu(blk.batch_norm(y)) + cur
        nxt.retain_grad()
        xs.append(nxt)
        cur = nxt
    pooled = F.max_pool2d(cur, 2).view(-1, 8 * 8 * model.n_chans1)
    if fc1_bf16:  # persistent engine: fc1 forward and its input-gradient use a bf16 copy of the weight
        w1 = model.fc1.weight
        w1r = w1 + (_bf(w1) - w1).detach()  # straight-through: dW is taken w.r.t. the fp32 master weight
        h = F.linear(pooled, w1r, model.fc1.bias)
    else:
        h = model.fc1(pooled)
    logits = model.fc2(torch.relu(h))
    loss = F.cross_entropy(logits, labels.long())
    for p in model.parameters():
        p.grad = None
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters()}
    res = {
        "loss": float(loss.detach()),
        "logits": logits.detach(),
        "grads": grads,
        "x": [t.detach() for t in xs],            # x_0 .. x_10 (NCHW)
        "y": [t.detach() for t in ys],            # y_0 .. y_9
        "dx": [t.grad.detach() if t.grad is not None else None for t in xs],
        "dy": [t.grad.detach() for t in ys],
    }
    if apply_sgd:
        with torch.no_grad():
            for p in model.parameters():
                p.add_(p.grad, alpha=-lr)
    return res


def nchw_to_nhwc(t: torch.Tensor) -> torch.Tensor:
    return t.permute(0, 2, 3, 1).contiguous()
