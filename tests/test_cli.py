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
