"""Entry points (reference main.py / main_no_ddp.py) on the CPU: output lines, checkpoint, fault injection."""
import os
import re
import subprocess
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ENV = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="2", CUDA_VISIBLE_DEVICES="", HIP_VISIBLE_DEVICES="")


def _run(args, timeout=400):
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=ENV, capture_output=True, text=True,
                          timeout=timeout)


def test_main_no_ddp_cpu_lines():
    r = _run(["main_no_ddp.py", "--synthetic", "640", "--epochs", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert lines[0] == "Training on device cpu."
    assert lines[1] == "10"  # len(train_loader) with batch 64
    assert re.fullmatch(r"Epoch 1, Training loss \d+\.\d+(e-?\d+)?", lines[2])
    assert re.fullmatch(r"training time: \d+\.\d{3} seconds", lines[3])


def test_main_gloo_two_ranks_checkpoint(tmp_path, port):
    ck = tmp_path / "birds_vs_airplanes.pt"
    r = _run(["main.py", "--backend", "gloo", "--world-size", "2", "--synthetic", "256", "--epochs", "1",
              "--max-steps", "2", "--engine", "torch", "--checkpoint-path", str(ck), "--port", str(port)])
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.count("Epoch 1, Training loss") == 2  # every rank prints its local mean (main.py:44)
    assert r.stdout.count("training time:") == 2
    sd = torch.load(str(ck), weights_only=True)
    assert len(sd) == 66
    assert int(sd["resblocks.0.batch_norm.num_batches_tracked"]) == 20  # 2 steps x 10 applications


def test_fault_injection_tears_down(tmp_path, port):
    r = _run(["main.py", "--backend", "gloo", "--world-size", "2", "--synthetic", "256", "--epochs", "1",
              "--max-steps", "4", "--engine", "torch", "--fail-at-step", "2", "--no-checkpoint", "--port", str(port),
              "--timeout", "60"])
    assert r.returncode != 0
    assert "injected failure at step 2" in r.stderr


def test_debug_flags_profile_check_sync_bucket(tmp_path, port):
    """--profile writes per-rank traces + kernel summaries; --check-sync asserts cross-rank parameter equality;
    --bucket-mb sets the generic path's bucket cap."""
    prof = tmp_path / "prof"
    r = _run(["main.py", "--backend", "gloo", "--world-size", "2", "--synthetic", "256", "--epochs", "1",
              "--max-steps", "2", "--engine", "torch", "--no-checkpoint", "--port", str(port), "--profile",
              str(prof), "--check-sync", "1", "--bucket-mb", "0.05"])
    assert r.returncode == 0, r.stderr[-3000:]
    for rk in (0, 1):
        assert (prof / f"trace_rank{rk}.json").stat().st_size > 0
        text = (prof / f"summary_rank{rk}.txt").read_text()
        assert "convolution" in text


def test_model_resnet50_flag(tmp_path):
    r = _run(["main_no_ddp.py", "--synthetic", "128", "--epochs", "1", "--max-steps", "1", "--model", "resnet50"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Training loss" in r.stdout


def _case_sync_check(rank, ws):
    import pytest as _pt
    import torch.nn as nn
    from distributeddataparallel_cifar10_amd.parallel import dist as pdist
    torch.manual_seed(0)
    m = nn.Linear(4, 4)
    pdist.assert_params_in_sync(m)  # identical on both ranks
    if rank == 1:
        with torch.no_grad():
            m.bias[0] += 1e-3
    with _pt.raises(RuntimeError, match="diverged"):
        pdist.assert_params_in_sync(m)


def test_check_sync_detects_divergence(port):
    from test_flat_ddp import _spawn
    _spawn(_case_sync_check, port, ws=2)


def test_train_loop_checks_comm_every_epoch():
    """train_loop calls the DDP wrapper's check_comm() at every epoch end (before any checkpoint), so a recorded
    all-reduce timeout stops training instead of silently diverging the ranks."""
    import pytest
    from distributeddataparallel_cifar10_amd.data.loader import DeviceLoader
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP
    from distributeddataparallel_cifar10_amd.train import TrainConfig, train_loop

    class Boom(RuntimeError):
        pass

    ddp = FlatBucketDDP(NetResDeep())
    calls = []

    def check():
        calls.append(1)
        raise Boom("peer timeout")

    ddp.check_comm = check
    data, labels = synthetic_cifar(64, seed=0)
    loader = DeviceLoader(data, labels, batch_size=32, world_size=1, rank=0, device="cpu")
    with pytest.raises(Boom):
        train_loop(ddp, loader, 0, TrainConfig(epochs=2, max_steps=1, checkpoint=False))
    assert calls == [1]


def test_resolve_engine_large_batch_falls_back():
    """The fused NetResDeep engine supports per-rank batch <= 64: auto picks the ops kernels above that, an
    explicit --engine fused raises a clear error instead of failing inside the native engine."""
    import pytest
    import torch
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.train import TrainConfig, resolve_engine
    cuda = torch.device("cuda", 0)
    m = NetResDeep()
    assert resolve_engine(TrainConfig(batch_size=64), cuda, m) == "fused"
    assert resolve_engine(TrainConfig(batch_size=128), cuda, m) == "ops"
    assert resolve_engine(TrainConfig(batch_size=128), torch.device("cpu"), m) == "torch"
    with pytest.raises(ValueError, match="batch-size"):
        resolve_engine(TrainConfig(batch_size=128, engine="fused"), cuda, m)


def test_bench_sets_dmabuf_ipc_mode():
    """bench.py (the driver's multi-GPU command) selects the dmabuf IPC mode itself, before any HIP call, so the
    xGMI all-reduce's IPC mappings work from a launcher environment without HSA_ENABLE_IPC_MODE_LEGACY; an
    explicit setting in the environment wins."""
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    code = "import os, bench; print(os.environ.get('HSA_ENABLE_IPC_MODE_LEGACY'))"
    env = dict(os.environ)
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "0", (r.stdout, r.stderr[-2000:])
    env["HSA_ENABLE_IPC_MODE_LEGACY"] = "1"
    r = subprocess.run([sys.executable, "-c", code], cwd=root, env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0 and r.stdout.strip() == "1", (r.stdout, r.stderr[-2000:])
