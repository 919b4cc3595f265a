"""CIFAR-10 readers (torchvision is not installed in this image) and the reference's input transform.

Reference behaviour (``main.py:53-58``, ``main_no_ddp.py:22-30``): ``datasets.CIFAR10(root, train=True,
download=False, transform=Compose([ToTensor(), Normalize(mean, std)]))`` over
``<root>/cifar-10-batches-py/data_batch_{1..5}`` (50,000 images; ``test_batch`` for train=False).

Here the whole split is read ONCE into a uint8 tensor ``[N, 3, 32, 32]`` (CHW, exactly the byte order of the
batch files) plus int64 labels.  The transform (``/255`` then ``(x - mean) / std``) is not applied on the host:
the engine's stem kernel applies it while gathering a batch (``csrc/common.h: norm_px``) and the torch path
applies it on the device (``normalize_u8``).

Two on-disk formats are accepted:
  * ``cifar-10-batches-py``: the pickled python batches torchvision reads.  They are opened with a RESTRICTED
    unpickler that only materialises dicts/lists/bytes/str/ints and plain numpy arrays (the only globals a CIFAR
    batch references); anything else in the stream raises ``pickle.UnpicklingError`` instead of running code.
  * ``cifar-10-batches-bin``: the binary distribution (1 label byte + 3072 pixel bytes per record), read with
    ``numpy.frombuffer`` -- no deserialisation at all.
"""
from __future__ import annotations

import io
import os
import pickle
from typing import Tuple

import numpy as np
import torch

# reference main.py:56-57
CIFAR10_MEAN = (0.4915, 0.4823, 0.4468)
CIFAR10_STD = (0.2470, 0.2435, 0.2616)

TRAIN_PY = [f"data_batch_{i}" for i in range(1, 6)]
TEST_PY = ["test_batch"]
TRAIN_BIN = [f"data_batch_{i}.bin" for i in range(1, 6)]
TEST_BIN = ["test_batch.bin"]

_ALLOWED_GLOBALS = {
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("_codecs", "encode"),
}


class _RestrictedUnpickler(pickle.Unpickler):
    """Unpickler that resolves only the numpy array-reconstruction globals a CIFAR batch uses."""

    def find_class(self, module, name):
        if (module, name) in _ALLOWED_GLOBALS:
            if module == "_codecs":
                import codecs
                return codecs.encode
            mod = __import__(module, fromlist=[name])
            return getattr(mod, name)
        raise pickle.UnpicklingError(f"CIFAR batch references forbidden global {module}.{name}")


def _load_py_batch(path: str) -> Tuple[np.ndarray, np.ndarray]:
    with open(path, "rb") as f:
        raw = f.read()
    d = _RestrictedUnpickler(io.BytesIO(raw), encoding="latin1").load()
    if not isinstance(d, dict):
        raise ValueError(f"{path}: not a CIFAR batch")
    data = d.get("data", d.get(b"data"))
    labels = d.get("labels", d.get(b"labels"))
    if data is None or labels is None:
        raise ValueError(f"{path}: missing data/labels")
    data = np.asarray(data, dtype=np.uint8).reshape(-1, 3, 32, 32)
    labels = np.asarray(labels, dtype=np.int64)
    if data.shape[0] != labels.shape[0]:
        raise ValueError(f"{path}: {data.shape[0]} images but {labels.shape[0]} labels")
    return data, labels


def _load_bin_batch(path: str) -> Tuple[np.ndarray, np.ndarray]:
    rec = np.fromfile(path, dtype=np.uint8)
    if rec.size % 3073:
        raise ValueError(f"{path}: size {rec.size} is not a multiple of 3073")
    rec = rec.reshape(-1, 3073)
    return rec[:, 1:].reshape(-1, 3, 32, 32).copy(), rec[:, 0].astype(np.int64)


def find_cifar10(root: str) -> Tuple[str, str]:
    """(format, directory) of a CIFAR-10 copy under `root` ("py" or "bin")."""
    for fmt, sub in (("py", "cifar-10-batches-py"), ("bin", "cifar-10-batches-bin")):
        d = os.path.join(root, sub)
        if os.path.isdir(d):
            return fmt, d
    raise FileNotFoundError(
        f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-py/ or cifar-10-batches-bin/; the reference "
        "also uses download=False). Use --synthetic for CIFAR-shaped synthetic data.")


def load_cifar10(root: str, train: bool = True) -> Tuple[torch.Tensor, torch.Tensor]:
    """uint8 images [N, 3, 32, 32] and int64 labels [N] of the train (50,000) or test (10,000) split."""
    fmt, d = find_cifar10(root)
    names = (TRAIN_PY if train else TEST_PY) if fmt == "py" else (TRAIN_BIN if train else TEST_BIN)
    loader = _load_py_batch if fmt == "py" else _load_bin_batch
    parts = [loader(os.path.join(d, n)) for n in names]
    data = np.concatenate([p[0] for p in parts])
    labels = np.concatenate([p[1] for p in parts])
    return torch.from_numpy(data), torch.from_numpy(labels)


def normalize_u8(x_u8: torch.Tensor) -> torch.Tensor:
    """ToTensor + Normalize of reference main.py:54-58 on a uint8 [N, 3, H, W] batch (any device)."""
    mean = torch.tensor(CIFAR10_MEAN, dtype=torch.float32, device=x_u8.device).view(1, 3, 1, 1)
    std = torch.tensor(CIFAR10_STD, dtype=torch.float32, device=x_u8.device).view(1, 3, 1, 1)
    return (x_u8.float() / 255.0 - mean) / std


def write_cifar10_bin(directory: str, data_u8: np.ndarray, labels: np.ndarray, train: bool = True,
                      n_files: int = 5) -> None:
    """Write a CIFAR-10 binary-format copy (tests / offline fixtures)."""
    os.makedirs(directory, exist_ok=True)
    names = TRAIN_BIN[:n_files] if train else TEST_BIN
    chunks = np.array_split(np.arange(len(labels)), len(names))
    for name, idx in zip(names, chunks):
        rec = np.concatenate([labels[idx].astype(np.uint8)[:, None], data_u8[idx].reshape(len(idx), -1)], axis=1)
        rec.astype(np.uint8).tofile(os.path.join(directory, name))
