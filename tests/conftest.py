"""Test configuration.

Markers:
  gpu  -- needs an MI355X (run with ``pytest -m gpu``); everything else runs on the CPU (``-m "not gpu"``).
  multigpu -- one rank per GPU across >= 2 devices (also ``gpu``; skipped on a 1-GPU box).
Multi-process tests use the gloo backend on 127.0.0.1.
"""
import os
import socket
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: requires an AMD Instinct GPU (MI355X, gfx950)")
    config.addinivalue_line("markers", "slow: long-running CPU test")
    config.addinivalue_line("markers", "multigpu: needs >= 2 MI355X on one node (also marked gpu; skips below 2)")


def free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.fixture
def port():
    return free_port()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a machine without a GPU (run with -m 'not gpu')")
    return torch.device("cuda", 0)
