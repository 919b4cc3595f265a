"""Diagnostic: the downsample residual-gradient link (ops/models.py _RES_LINK) against the written path -- order of
the fused conv-BN backward calls and per-parameter gradient differences (ResNet [1, 1, 1, 1]: downsample blocks
only; [2, 1, 1, 1] also has an identity block)."""
import copy
import sys
import os

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    from distributeddataparallel_cifar10_amd.ops import OpsModel, cross_entropy
    from distributeddataparallel_cifar10_amd.ops import functional as F
    from distributeddataparallel_cifar10_amd.ops import models as M_
    dev = torch.device("cuda", 0)
    for layers in ([1, 1, 1, 1], [2, 1, 1, 1]):
        torch.manual_seed(0)
        net = ResNet(layers, num_classes=10, zero_init_residual=False).to(dev)
        other = copy.deepcopy(net)
        x = torch.randn(8, 3, 192, 192, device=dev)
        y = torch.randint(0, 10, (8,), device=dev)
        res = []
        for m, on in ((net, True), (other, False)):
            M_._RES_LINK = on
            F._BWD_TRACE = []
            cross_entropy(OpsModel(m)(x), y).backward()
            res.append((F._BWD_TRACE, [p.grad.clone() for p in m.parameters()]))
        F._BWD_TRACE = None
        print(f"layers {layers}: order equal: {[t[0] for t in res[0][0]] == [t[0] for t in res[1][0]]}")
        print("  on :", res[0][0])
        print("  off:", res[1][0])
        for (n, _), g1, g2 in zip(net.named_parameters(), res[0][1], res[1][1]):
            if not torch.equal(g1, g2):
                d = (g1 - g2).abs().max().item()
                print(f"  {n:40s} max|diff| {d:.3e}  rel {(g1 - g2).norm().item() / max(g2.norm().item(), 1e-30):.3e}")
    M_._RES_LINK = True


if __name__ == "__main__":
    main()
