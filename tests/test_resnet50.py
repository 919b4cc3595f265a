"""ResNet-50 family (BASELINE extension config) on the generic data-parallel path, small inputs on CPU."""
import torch
import torch.nn.functional as F

from distributeddataparallel_cifar10_amd.models.resnet50 import resnet50, resnet101
from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD


def test_resnet50_shapes_and_params():
    m = resnet50()
    assert sum(p.numel() for p in m.parameters()) == 25_557_032  # the standard ResNet-50 count
    assert m(torch.randn(2, 3, 64, 64)).shape == (2, 1000)
    assert sum(p.numel() for p in resnet101().parameters()) == 44_549_160


def test_flat_sgd_momentum_matches_torch():
    torch.manual_seed(0)
    a = resnet50(num_classes=10)
    b = resnet50(num_classes=10)
    b.load_state_dict(a.state_dict())
    ddp = FlatBucketDDP(a, bucket_cap_mb=8.0)
    opt_a = FlatSGD(ddp, lr=0.05, momentum=0.9, weight_decay=1e-4)
    opt_b = torch.optim.SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=1e-4)
    x = torch.randn(2, 3, 32, 32)
    y = torch.tensor([1, 7])
    for _ in range(2):
        for model, opt in ((ddp, opt_a), (b, opt_b)):
            loss = F.cross_entropy(model(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-4), n
    assert len(ddp.buckets) >= 3  # 25.5 M params -> several buckets
