"""Reference-compatible import path: ``from model.resnet import NetResDeep`` (reference ``main.py:7``).

The implementation lives in the framework package (``distributeddataparallel_cifar10_amd.models.netresdeep``).
"""
from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep, ResBlock  # noqa: F401

__all__ = ["NetResDeep", "ResBlock"]
