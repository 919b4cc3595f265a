"""Data layer: DistributedSampler parity, CIFAR-10 readers (safe), device loader lengths."""
import io
import os
import pickle

import numpy as np
import pytest
import torch
from torch.utils.data.distributed import DistributedSampler

from distributeddataparallel_cifar10_amd.data.cifar import (CIFAR10_MEAN, CIFAR10_STD, load_cifar10, normalize_u8,
                                                            write_cifar10_bin)
from distributeddataparallel_cifar10_amd.data.loader import DeviceLoader
from distributeddataparallel_cifar10_amd.data.sampler import batches_per_epoch, distributed_indices
from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar


@pytest.mark.parametrize("n,ws", [(50000, 1), (50000, 2), (50000, 8), (101, 4), (10, 3)])
@pytest.mark.parametrize("drop_last", [False, True])
def test_sampler_bit_identical(n, ws, drop_last):
    for rank in range(ws):
        for epoch in (0, 3):
            ref = DistributedSampler(range(n), num_replicas=ws, rank=rank, drop_last=drop_last)
            ref.set_epoch(epoch)
            ours = distributed_indices(n, ws, rank, epoch=epoch, drop_last=drop_last)
            assert ours.tolist() == list(iter(ref))


def test_batches_per_epoch_table():
    # per-rank batches/epoch at bs=32
    for ws, nb in ((1, 1563), (2, 782), (4, 391), (8, 196)):
        assert batches_per_epoch(len(distributed_indices(50000, ws, 0)), 32) == nb
    assert batches_per_epoch(50000, 64) == 782  # main_no_ddp.py prints 782


def test_cifar_bin_roundtrip(tmp_path):
    data, labels = synthetic_cifar(50, seed=3)
    write_cifar10_bin(str(tmp_path / "cifar-10-batches-bin"), data.numpy(), labels.numpy())
    d2, l2 = load_cifar10(str(tmp_path), train=True)
    assert torch.equal(d2, data) and torch.equal(l2, labels)


def _write_py_batches(root, data, labels):
    d = os.path.join(root, "cifar-10-batches-py")
    os.makedirs(d)
    parts = np.array_split(np.arange(len(labels)), 5)
    for i, idx in enumerate(parts, 1):
        with open(os.path.join(d, f"data_batch_{i}"), "wb") as f:
            pickle.dump({b"data": data[idx].reshape(len(idx), -1), b"labels": labels[idx].tolist()}, f)


def test_cifar_py_restricted_unpickler(tmp_path):
    data, labels = synthetic_cifar(40, seed=4)
    _write_py_batches(str(tmp_path), data.numpy(), labels.numpy())
    d2, l2 = load_cifar10(str(tmp_path), train=True)
    assert torch.equal(d2, data) and torch.equal(l2, labels)


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_cifar_py_rejects_code(tmp_path):
    d = tmp_path / "cifar-10-batches-py"
    d.mkdir()
    for i in range(1, 6):
        with open(d / f"data_batch_{i}", "wb") as f:
            pickle.dump({b"data": _Evil(), b"labels": []}, f)
    with pytest.raises(pickle.UnpicklingError):
        load_cifar10(str(tmp_path))


def test_missing_dataset_message(tmp_path):
    with pytest.raises(FileNotFoundError, match="--synthetic"):
        load_cifar10(str(tmp_path))


def test_normalize_matches_totensor_normalize():
    x = torch.randint(0, 256, (2, 3, 4, 4), dtype=torch.uint8)
    exp = (x.float() / 255 - torch.tensor(CIFAR10_MEAN).view(1, 3, 1, 1)) / torch.tensor(CIFAR10_STD).view(1, 3, 1, 1)
    assert torch.allclose(normalize_u8(x), exp)


def test_device_loader_order_and_len():
    data, labels = synthetic_cifar(100, seed=0)
    ld = DeviceLoader(data, labels, batch_size=32, world_size=2, rank=1)
    assert len(ld) == 2  # 50 local samples -> 32 + 18
    idx = distributed_indices(100, 2, 1)
    batches = list(ld)
    assert [b[0].shape[0] for b in batches] == [32, 18]
    assert torch.equal(batches[1][1], labels[idx[32:]])
    assert torch.allclose(batches[0][0], normalize_u8(data[idx[:32]]))
    # reference never calls set_epoch: same order every epoch unless opted in
    ld.set_epoch(5)
    assert np.array_equal(ld.indices(), idx)
    ld2 = DeviceLoader(data, labels, batch_size=32, world_size=2, rank=1, set_epoch=True)
    ld2.set_epoch(5)
    assert not np.array_equal(ld2.indices(), idx)
