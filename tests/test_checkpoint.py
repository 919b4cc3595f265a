"""Checkpoint format parity (reference main.py:45) and safe loading."""
import os

import torch

from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP
from distributeddataparallel_cifar10_amd.runtime.engine import bind_flat_parameters
from distributeddataparallel_cifar10_amd.utils.checkpoint import (CHECKPOINT_NAME, export_state_dict, load_checkpoint,
                                                                  save_checkpoint)


def test_rank0_only_atomic_write(tmp_path):
    m = NetResDeep()
    path = str(tmp_path / "data" / CHECKPOINT_NAME)
    assert save_checkpoint(m, path, rank=1) is None and not os.path.exists(path)
    assert save_checkpoint(m, path, rank=0, meta={"epoch": 10, "step": 5}) == path
    assert not [f for f in os.listdir(tmp_path / "data") if ".tmp" in f]
    sd = torch.load(path, weights_only=True)
    assert len(sd) == 66 and all(not k.startswith("module.") for k in sd)
    assert sd["resblocks.0.conv.weight"].data_ptr() == sd["resblocks.7.conv.weight"].data_ptr()  # aliasing kept
    assert sd["conv1.weight"].dtype == torch.float32


def test_wrapped_model_saves_unprefixed_keys(tmp_path):
    m = NetResDeep()
    w = FlatBucketDDP(m)  # ws=1: no process group needed
    path = str(tmp_path / CHECKPOINT_NAME)
    save_checkpoint(w, path)
    sd = torch.load(path, weights_only=True)
    assert set(sd) == set(m.state_dict())


def test_roundtrip_into_reference_model(tmp_path):
    torch.manual_seed(0)
    m = NetResDeep()
    bind_flat_parameters(m, "cpu")  # engine-style flat views must export plain tensors
    with torch.no_grad():
        m.fc1.weight.add_(1.0)
        m.resblocks[0].batch_norm.running_mean.fill_(0.25)
        m.resblocks[0].batch_norm.num_batches_tracked.fill_(30)
    path = str(tmp_path / CHECKPOINT_NAME)
    save_checkpoint(m, path, meta={"epoch": 3, "step": 99})
    ref = NetResDeep()
    meta = load_checkpoint(ref, path, strict=True)
    assert meta == {"epoch": 3, "step": 99}
    for k, v in m.state_dict().items():
        assert torch.equal(ref.state_dict()[k], v), k


def test_export_is_cpu_and_detached():
    m = NetResDeep()
    sd = export_state_dict(m)
    assert all(t.device.type == "cpu" and not t.requires_grad for t in sd.values())


def test_trace_range_nests_and_never_fails():
    from distributeddataparallel_cifar10_amd.utils.trace import trace_range
    with trace_range("outer"):
        with trace_range("inner"):
            x = 1 + 1
    assert x == 2
