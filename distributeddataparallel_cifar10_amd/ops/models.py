"""Model forwards on the ops layer (HIP kernels for every layer), sharing the parameters of the torch modules.

``OpsModel(model)`` wraps a ``NetResDeep`` (reference ``model/resnet.py``) or a ResNet (``models/resnet50.py``)
without copying anything: the wrapped module's ``nn.Parameter``s and BN buffers are the ones the kernels read
and the optimizer updates, so ``state_dict()`` is unchanged.  The forward takes the usual NCHW fp32 batch,
switches to channels-last bf16 once, and runs:

* NetResDeep (reference ``model/resnet.py:15-37``): conv1 + bias + ReLU fused in the GEMM epilogue -> 2x2 max
  pool -> 10 x [3x3 conv (im2col + MFMA GEMM) -> BN + ReLU + skip fused (res_mode 1)] -> max pool -> fc1 + ReLU
  -> fc2 (fp32 logits).  fc1's columns are permuted from the reference's NCHW flatten order to NHWC.
* ResNet-50/101: stem 7x7/2 conv -> BN + ReLU + 3x3/2 max pool (one fused pass) -> bottlenecks (1x1, 3x3, 1x1 convs, each BN
  fused with its ReLU; the last one with the residual add before the ReLU, res_mode 2) -> global average pool
  -> fc.  The 7x7/2 stem runs as a 4x4 stride-1 conv over a space-to-depth copy of the input (K 256 instead of
  392).  The bf16 (and fp8) GEMM operands of all convolutions are rebuilt from the fp32 weights by one
  ``WeightPack`` launch per step, and the conv / BN parameter gradients are written straight into the flat
  gradient buffer of ``FlatBucketDDP`` when the model is wrapped in it (``functional.grad_sink``).
  With ``fp8=True`` the 3x3 convolutions (implicit GEMM over an fp8 NHWC copy of the input), fc, and optionally
  the 1x1 convolutions (``DCA_FP8_MIN_CIN``) run their forward GEMM in fp8 e4m3 on the MX-scaled MFMA (fp8 rate):
  weights are quantised per step (WeightPack, device-side amax); activations are emitted in
  fp8 directly by the producing BN kernel with delayed scaling (previous step's amax, ``functional.Fp8Delayed``);
  gradients and the backward stay bf16 (BASELINE config 5).
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn

from . import functional as F

# DCA_OPS_MASKED_JOIN=0: bn3's backward writes the identity gradient dout * mask as before (A/B comparisons)
_MASKED_JOIN = os.environ.get("DCA_OPS_MASKED_JOIN", "1") != "0"
_RES_LINK = os.environ.get("DCA_OPS_RES_LINK", "1") != "0"  # downsample blocks: the residual gradient over a link


def _is_netresdeep(m: nn.Module) -> bool:
    return hasattr(m, "resblocks") and hasattr(m, "fc1") and hasattr(m, "fc2")


class OpsModel(nn.Module):
    def __init__(self, model: nn.Module, fp8: bool = False):
        super().__init__()
        self.module = model
        self.fp8 = fp8
        self.kind = "netresdeep" if _is_netresdeep(model) else "resnet"
        self._pack = None
        self._s2d = None

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        if self.kind == "netresdeep":
            h = x.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous()  # NCHW fp32 -> NHWC bf16
            return self._netresdeep(h)
        return self._resnet(self.begin(x))

    def begin(self, x: torch.Tensor) -> torch.Tensor:
        """Per-step entry of a ResNet-family forward: NCHW fp32 input -> NHWC bf16 (the 3-channel input
        zero-padded to 8 channels so the 7x7 stem is an implicit GEMM), every conv's GEMM operands packed from
        this step's fp32 weights (one launch), every BN's num_batches_tracked += 1 (one launch, training only).
        Models that compose the stages themselves (``apps/ppe.py``'s ROI head) call this, then ``stem`` /
        ``blocks`` / ``head``."""
        if self._pack is None:
            convs = [m for m in self.module.modules() if isinstance(m, nn.Conv2d)]
            # the stem (the first conv: ResNet conv1, the PPE model's stem[0]) as a space-to-depth 4x4 conv when it
            # is 7x7/2/3 over <= 4 channels (DCA_OPS_STEM_S2D=0: the 8-channel NHWC 7x7 implicit GEMM).  Decided
            # here, at the first step: an input that requires grad (no input gradient through the s2d stem) keeps
            # the regular 7x7 path for the model's lifetime
            self._s2d = convs[0] if convs and self.kind == "resnet" and F.stem_s2d_ok(convs[0]) and \
                not x.requires_grad and os.environ.get("DCA_OPS_STEM_S2D", "1") != "0" else None
            self._pack = F.WeightPack(convs, [c for c in convs if self._fp8_ok(c)],
                                      [self._s2d] if self._s2d is not None else [])
            self._bns = [m for m in self.module.modules()
                         if isinstance(m, nn.BatchNorm2d) and m.track_running_stats]
            for m in self._bns:
                m._dca_counted = True
            self._nbt_key = None
        if self._s2d is not None:
            if x.requires_grad:
                raise NotImplementedError("OpsModel: the first step's input did not require grad, so the stem "
                                          "runs space-to-depth (no input gradient); build the model with a "
                                          "requires_grad input first, or set DCA_OPS_STEM_S2D=0")
            h = F.nchw_to_s2d16(x.detach().float())  # one kernel: the stem's space-to-depth operand
        elif x.shape[1] <= 8 and x.dtype == torch.float32 and not x.requires_grad:
            h = F.nchw_to_nhwc8(x)  # one kernel
        else:
            h = x.permute(0, 2, 3, 1)
            if h.shape[-1] % 8:
                h = torch.nn.functional.pad(h, (0, 8 - h.shape[-1] % 8))
            h = h.to(torch.bfloat16).contiguous()
        self._pack.pack()  # every conv's bf16 / fp8 GEMM operands from this step's fp32 weights: one launch
        if self.training and self.module.training and self._bns:  # each BN runs once per step: one launch
            key = tuple(m.num_batches_tracked.data_ptr() for m in self._bns)
            if key != self._nbt_key:  # the counters moved (e.g. into FlatBucketDDP's flat int64 buffer)
                self._nbt_ptrs = torch.tensor(list(key), dtype=torch.int64).to(h.device)
                self._nbt_key = key
            F.add_one_i64(self._nbt_ptrs, len(key))
        return h

    # reference model/resnet.py:15-22, 33-37
    def _netresdeep(self, h):
        m = self.module
        h = F.conv2d(h, m.conv1.weight, m.conv1.bias, stride=1, pad=1, relu=True)
        h = F.max_pool2d(h, 2)
        for blk in m.resblocks:  # relu(bn(conv(x))) + x, BN statistics from the conv GEMM's epilogue
            h = F.conv_bn_act(h, blk.conv, blk.batch_norm, r=h, relu=True, res_mode=1)
        h = F.max_pool2d(h, 2)
        n, hh, ww, c = h.shape
        flat = h.reshape(n, hh * ww * c)
        w1 = m.fc1.weight.view(-1, c, hh, ww).permute(0, 2, 3, 1).reshape(m.fc1.weight.shape[0], -1)
        z = F.linear(flat, w1, m.fc1.bias, relu=True, out_dtype=torch.bfloat16)
        return F.linear(z, m.fc2.weight, m.fc2.bias, out_dtype=torch.float32)

    # fp8 pays where the GEMM is MFMA-bound: the 3x3 convolutions (K = 9 Cin).  For the 1x1 convolutions the fp8
    # copy the producer must write costs more than the faster GEMM saves (measured at batch 256: 1x1 fp8 from
    # Cin >= 256 / 512 / 1024 / never -> 7659 / 7681 / 7729 / 7763 img/s, bf16 7708), so they stay bf16 unless
    # DCA_FP8_MIN_CIN (>= 128) asks for them.
    FP8_MIN_CIN = int(os.environ.get("DCA_FP8_MIN_CIN", "0")) or None

    def _fp8_ok(self, conv) -> bool:
        """fp8 forward GEMM for 1x1 stride-1 convolutions with K = Cin >= FP8_MIN_CIN (the fp8 K-tile is 128
        deep) and for 3x3 convolutions (K = 9 Cin, implicit GEMM over the input's fp8 copy; Cin % 16 == 0)."""
        if not self.fp8:
            return False
        if conv.kernel_size == (3, 3):
            return conv.in_channels % 16 == 0 and conv.in_channels >= 64
        return (self.FP8_MIN_CIN is not None and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
                and conv.padding == (0, 0) and conv.in_channels >= max(128, self.FP8_MIN_CIN))

    def _state(self, conv):
        if not self._fp8_ok(conv):
            return None
        if not hasattr(self, "_fp8"):
            self._fp8 = {}
        return self._fp8.setdefault(id(conv), F.Fp8Delayed())

    def _conv_bn(self, h, conv, bn, relu=True, r=None, consumer=None, x_join=None, r_join=None, res_in=None,
                 pool=False):
        # every ResNet conv / BN is applied once per step: gradients may go straight into the flat DDP buffer
        return F.conv_bn_act(h, conv, bn, r=r, relu=relu, fp8=self._fp8_ok(conv), fp8_state=self._state(conv),
                             emit=self._state(consumer) if consumer is not None else None,
                             packed=self._pack.get(conv), direct_grads=True, x_join=x_join, r_join=r_join,
                             res_in=res_in, pool=pool)

    def stem(self, h, conv, bn):
        """7x7/2 conv -> BN + ReLU -> 3x3/2 max pool (torchvision ResNet stem).  ``h`` is what ``begin`` returned:
        for the space-to-depth stem its [N, Ho + 3, Wo + 3, 16] operand (the conv then runs as 4x4 / 1)."""
        if self._s2d is not None and conv is not self._s2d:
            raise ValueError("OpsModel.stem: begin() prepared the space-to-depth input of this model's first conv")
        return self._conv_bn(h, conv, bn, pool=True)  # BN + ReLU + pool in one pass each way (F.bn_pool_ok)

    def blocks(self, h, blocks):
        """Bottleneck blocks in sequence over NHWC bf16 ``h``."""
        blocks = list(blocks)
        for i, b in enumerate(blocks):
            nxt = blocks[i + 1].conv1 if i + 1 < len(blocks) else None
            # the block input feeds conv1 and the identity / downsample path: one shared gradient buffer
            c1 = b.conv1
            # identity blocks whose conv1 dgrad runs on the stream GEMM (1x1, K = conv1 width <= 256, >= 16384
            # pixels): bn3's backward skips writing dout * mask, the dgrad epilogue reads dout and the mask
            # (layer 3, K = 256: 83.2 us on the stream kernel with the masked source against 83.8 us on glds with
            # a written C_old, bench/gemm_beta_k256.py)
            defer = (b.downsample is None and _MASKED_JOIN and tuple(c1.kernel_size) == (1, 1)
                     and tuple(c1.stride) == (1, 1) and c1.out_channels <= 256
                     and h.shape[0] * h.shape[1] * h.shape[2] >= 16384)
            join = F.GradJoin(2, defer_ok=defer)
            rlink = F.ResidualLink() if b.downsample is not None and _MASKED_JOIN and _RES_LINK else None
            if b.downsample is None:
                idt = h
            else:
                idt = self._conv_bn(h, b.downsample[0], b.downsample[1], relu=False, x_join=join, res_in=rlink)
            out = self._conv_bn(h, b.conv1, b.bn1, x_join=join, consumer=b.conv2)
            out = self._conv_bn(out, b.conv2, b.bn2, consumer=b.conv3)
            h = self._conv_bn(out, b.conv3, b.bn3, relu=True, r=idt, consumer=nxt,
                              r_join=join if b.downsample is None else rlink)  # relu(bn3(conv3) + identity)
        return h

    def head(self, h, fc):
        """Global average pool -> fc (fp32 logits)."""
        feat = F.global_avg_pool(h, out_dtype=torch.bfloat16)  # the fc operand directly (no cast pass)
        return F.linear(feat, fc.weight, fc.bias, out_dtype=torch.float32, fp8=self.fp8)

    def _resnet(self, h):
        m = self.module
        h = self.stem(h, m.conv1, m.bn1)
        h = self.blocks(h, [b for stage in (m.layer1, m.layer2, m.layer3, m.layer4) for b in stage])
        return self.head(h, m.fc)
