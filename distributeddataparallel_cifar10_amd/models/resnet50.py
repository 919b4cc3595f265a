"""ResNet-50 (bottleneck v1.5: stride on the 3x3 conv), written from scratch (torchvision is not installed).

BASELINE.json lists "ResNet-50 on synthetic 3x224x224 DDP 8xMI355X" as an extension configuration of this
framework.  The reference's second application (``ppe_main_ddp.py``) fine-tunes a ResNet-101 under the same DDP
wrapper; its model file is missing from the reference, so the ResNet family here is defined
from the standard architecture: stem 7x7/2 conv + 3x3/2 max-pool, stages of [3, 4, 6, 3] (ResNet-50) or
[3, 4, 23, 3] (ResNet-101) bottlenecks with expansion 4, global average pool, fc.

Training runs through the generic data-parallel path (``parallel/flat_ddp.py``: flat buffers, bucketed async
all-reduce overlapped with backward, fused flat SGD) with bf16 autocast and channels-last activations.
"""
from __future__ import annotations

from typing import List, Optional

import torch
import torch.nn as nn


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, in_ch: int, width: int, stride: int = 1, downsample: Optional[nn.Module] = None):
        super().__init__()
        out_ch = width * self.expansion
        self.conv1 = nn.Conv2d(in_ch, width, 1, bias=False)
        self.bn1 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, out_ch, 1, bias=False)
        self.bn3 = nn.BatchNorm2d(out_ch)
        self.relu = nn.ReLU(inplace=True)
        self.downsample = downsample

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        idt = x if self.downsample is None else self.downsample(x)
        out = self.relu(self.bn1(self.conv1(x)))
        out = self.relu(self.bn2(self.conv2(out)))
        out = self.bn3(self.conv3(out))
        return self.relu(out + idt)


class ResNet(nn.Module):
    def __init__(self, layers: List[int], num_classes: int = 1000, zero_init_residual: bool = True):
        super().__init__()
        self.in_ch = 64
        self.conv1 = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.bn1 = nn.BatchNorm2d(64)
        self.relu = nn.ReLU(inplace=True)
        self.maxpool = nn.MaxPool2d(3, stride=2, padding=1)
        self.layer1 = self._stage(64, layers[0], 1)
        self.layer2 = self._stage(128, layers[1], 2)
        self.layer3 = self._stage(256, layers[2], 2)
        self.layer4 = self._stage(512, layers[3], 2)
        self.avgpool = nn.AdaptiveAvgPool2d(1)
        self.fc = nn.Linear(512 * Bottleneck.expansion, num_classes)
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)

    def _stage(self, width: int, blocks: int, stride: int) -> nn.Sequential:
        out_ch = width * Bottleneck.expansion
        down = None
        if stride != 1 or self.in_ch != out_ch:
            down = nn.Sequential(nn.Conv2d(self.in_ch, out_ch, 1, stride=stride, bias=False), nn.BatchNorm2d(out_ch))
        mods = [Bottleneck(self.in_ch, width, stride, down)]
        self.in_ch = out_ch
        mods += [Bottleneck(out_ch, width) for _ in range(1, blocks)]
        return nn.Sequential(*mods)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        x = self.maxpool(self.relu(self.bn1(self.conv1(x))))
        x = self.layer4(self.layer3(self.layer2(self.layer1(x))))
        return self.fc(torch.flatten(self.avgpool(x), 1))


def resnet50(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 6, 3], num_classes)


def resnet101(num_classes: int = 1000) -> ResNet:
    return ResNet([3, 4, 23, 3], num_classes)
