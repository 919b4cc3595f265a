"""NetResDeep parity with reference model/resnet.py (structure, sharing, state_dict, init, BN bookkeeping)."""
import torch
import torch.nn.functional as F

from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep, ResBlock
from model.resnet import NetResDeep as ShimNetResDeep


def test_import_path_matches_reference():
    assert ShimNetResDeep is NetResDeep  # `from model.resnet import NetResDeep` (reference main.py:7)


def test_shared_block_and_param_count():
    m = NetResDeep()
    assert len({id(b) for b in m.resblocks}) == 1  # ONE ResBlock applied 10x (model/resnet.py:10-11)
    params = list(m.parameters())
    assert len(params) == 9
    assert sum(p.numel() for p in params) == 76074


def test_state_dict_keys_and_aliasing():
    m = NetResDeep()
    sd = m.state_dict()
    assert len(sd) == 66
    storages = {t.untyped_storage().data_ptr() for t in sd.values()}
    assert len(storages) == 12
    assert sd["resblocks.0.conv.weight"].data_ptr() == sd["resblocks.9.conv.weight"].data_ptr()
    assert sd["resblocks.3.batch_norm.num_batches_tracked"].dtype == torch.int64


def test_init_distributions():
    torch.manual_seed(0)
    b = ResBlock(32)
    assert torch.all(b.batch_norm.weight == 0.5) and torch.all(b.batch_norm.bias == 0)
    assert b.conv.bias is None
    std = b.conv.weight.std().item()
    assert abs(std - (2.0 / (32 * 9)) ** 0.5) < 0.01  # kaiming_normal_(relu)


def test_forward_matches_functional_definition():
    torch.manual_seed(1)
    m = NetResDeep()
    x = torch.randn(4, 3, 32, 32)
    out = m(x)
    assert out.shape == (4, 10)
    # explicit re-statement of reference model/resnet.py:15-22, 33-37
    blk = m.resblocks[0]
    ref = NetResDeep()
    ref.load_state_dict(m.state_dict())
    h = F.max_pool2d(torch.relu(ref.conv1(x)), 2)
    for _ in range(10):
        h = torch.relu(ref.resblocks[0].batch_norm(ref.resblocks[0].conv(h))) + h
    h = F.max_pool2d(h, 2).view(-1, 2048)
    exp = ref.fc2(torch.relu(ref.fc1(h)))
    assert torch.allclose(out, exp, atol=1e-5)
    assert int(blk.batch_norm.num_batches_tracked) == 10  # +1 per application


def test_reference_state_dict_loads_deALIASED():
    m = NetResDeep()
    sd = {k: v.clone() for k, v in m.state_dict().items()}  # 66 independent copies
    m2 = NetResDeep()
    m2.load_state_dict(sd, strict=True)
    assert torch.equal(m2.resblocks[5].conv.weight, m.resblocks[0].conv.weight)
