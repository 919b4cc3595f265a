"""Cross-device data parallelism: one rank per GPU on a multi-GPU MI355X node (the ``multigpu`` tests skip below
2 devices, so the 1-GPU tier collects and skips them; on an 8-GPU node they run unchanged).

* the fused trainer's DDP step against the single-process simulation of reference DDP (bf16 and fp32), with the
  slabs / flags crossing xGMI (comm="xgmi") and with the graph-captured RCCL all-reduce (comm="rccl");
  bitwise-equal parameters on all ranks;
* the driver's exact command (``python bench.py --gpus N``, ranks self-launched) and its torchrun form, both
  all-reduce paths, plus ``--sweep 1,2,N`` with its scaling-efficiency summary;
* ResNet (ops kernels) under FlatBucketDDP + XgmiComm against the host-averaged per-rank reference.

The ``shared`` variants run the same commands with every rank on GPU 0 (DCA_BENCH_SHARE_GPU=1: gloo process
group, the engine's xGMI path between ranks on one device), so the 1-GPU tier exercises them every round.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpu() -> int:
    return torch.cuda.device_count()


needs2 = [pytest.mark.multigpu, pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")]


def _json_lines(out: str) -> list:
    return [json.loads(ln) for ln in out.splitlines() if ln.startswith("{")]


def _bench(args, shared=False, timeout=420):
    env = dict(os.environ, DCA_XGMI_TIMEOUT_S="30")
    env.pop("DCA_BENCH_SHARE_GPU", None)
    if shared:  # ranks sharing GPU 0: one hardware queue each (tests/_ranks.py)
        env["DCA_BENCH_SHARE_GPU"] = "1"
        env["GPU_MAX_HW_QUEUES"] = "1"
    r = subprocess.run([sys.executable, *args], cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stderr[-4000:]
    return _json_lines(r.stdout)


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
@pytest.mark.parametrize("comm", ["xgmi", "rccl"])
@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_ddp_engine_cross_device(gpu, port, comm, dtype):
    from test_ddp_engine_gpu import _xgmi_worker
    ws = min(_ngpu(), 8)
    from _ranks import spawn_ranks
    spawn_ranks(_xgmi_worker, ws, lambda r: (r, ws, port, dtype, True), dict(comm=comm, own_device=True), shared=False)


def _check_bench_line(out, n, allreduce=None, batch=32):
    assert out["n_gpus"] == n and out["value"] > 0 and out["loss_finite"], out
    assert out["config"]["parallelism"] == f"dp{n}" and out["config"]["global_batch"] == batch * n
    if allreduce is not None:
        assert out["allreduce"] == allreduce, out
    if n > 1 and out["allreduce"] == "xgmi":
        assert len(out["allreduce_us_per_step"]) == n
    assert out["fp32_value"] > 0 and out["fp32_loss_finite"] and out["fp32_mode"] in ("3xbf16", "fp32-mfma")


@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_bench_driver_command(gpu):
    """The driver's command verbatim: ``python bench.py --gpus N --steps K --warmup W`` (bench.py spawns the N
    ranks itself); bf16 value plus the fp32 (reference precision) timing of the same invocation."""
    n = min(_ngpu(), 8)
    lines = _bench(["bench.py", "--gpus", str(n), "--steps", "48", "--warmup", "16"])
    assert len(lines) == 1, lines
    _check_bench_line(lines[0], n)


@pytest.mark.parametrize("allreduce", ["xgmi", "rccl"])
@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_bench_torchrun_one_rank_per_gpu(gpu, port, allreduce):
    n = min(_ngpu(), 8)
    lines = _bench(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
                    "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n), "--steps", "48",
                    "--warmup", "16", "--allreduce", allreduce])
    assert len(lines) == 1, lines
    _check_bench_line(lines[0], n, allreduce)


@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_bench_sweep(gpu):
    """``--sweep 1,2,N``: one fresh rank group per N and the scaling summary the headline metric asks for."""
    n = min(_ngpu(), 8)
    ns = sorted({1, 2, n})
    lines = _bench(["bench.py", "--sweep", ",".join(map(str, ns)), "--steps", "48", "--warmup", "16", "--no-fp32"],
                   timeout=900)
    per_n, summary = lines[:-1], lines[-1]
    assert [ln["n_gpus"] for ln in per_n] == ns and all(ln["loss_finite"] for ln in per_n)
    assert set(summary["scaling_efficiency"]) == {str(k) for k in ns}
    assert summary["scaling_efficiency"]["1"] == 1.0
    assert all(0.0 < v for v in summary["scaling_efficiency"].values())


@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_resnet_flat_ddp_xgmi_cross_device(gpu, port):
    """ResNet (ops kernels, small batch / image) under FlatBucketDDP + XgmiComm, one rank per GPU, against the
    per-rank reference with host-averaged gradients."""
    from test_xgmi_comm_gpu import _ops_ddp_worker, _spawn
    _spawn(_ops_ddp_worker, min(_ngpu(), 8), port, own_device=True)


@pytest.mark.multigpu
@pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")
def test_resnet50_bench_self_launch(gpu):
    """bench/resnet50.py --gpus N spawns one rank per GPU itself (FlatBucketDDP over xGMI, ops kernels); small
    batch / image so it finishes quickly."""
    n = min(_ngpu(), 8)
    lines = _bench(["bench/resnet50.py", "--gpus", str(n), "--batch", "16", "--image", "64", "--steps", "3",
                    "--warmup", "1"], timeout=600)
    assert len(lines) == 1, lines
    assert lines[0]["n_gpus"] == n and lines[0]["value"] > 0 and lines[0]["loss"] == lines[0]["loss"]


# ---- shared-GPU rehearsals of the same commands (run on the 1-GPU tier) ----------------------------------------
def test_bench_driver_command_shared_gpu(gpu):
    """``python bench.py --gpus 2`` with both ranks on GPU 0: self-launch, gloo rendezvous, the engine's xGMI
    gradient exchange between the ranks, slowest-rank timing and the fp32 second timing.  Per-rank batch 16: two
    batch-32 grids (2 x 128 step workgroups) would fill the device exactly, which the co-residency rule refuses."""
    lines = _bench(["bench.py", "--gpus", "2", "--batch", "16", "--steps", "32", "--warmup", "8"], shared=True)
    assert len(lines) == 1, lines
    _check_bench_line(lines[0], 2, "xgmi", batch=16)


def test_bench_sweep_shared_gpu(gpu):
    lines = _bench(["bench.py", "--sweep=1,2", "--batch", "16", "--steps", "32", "--warmup", "8", "--no-fp32"], shared=True,
                   timeout=600)
    per_n, summary = lines[:-1], lines[-1]
    assert [ln["n_gpus"] for ln in per_n] == [1, 2] and all(ln["loss_finite"] for ln in per_n)
    assert set(summary["scaling_efficiency"]) == {"1", "2"}


def test_bench_driver_command_shared_gpu_8_ranks(gpu):
    """``python bench.py --gpus 8`` -- the driver's N=8 command -- rehearsed with all 8 ranks on GPU 0 at a per-rank
    batch of 4 (each rank's 16-workgroup step grid at half its 256 / 8 CU budget: at batch 8 the grid filled the
    budget exactly and a rank's BN exchange once timed out while a peer's kernels held CUs): self-launch of 8 ranks,
    the engine's xGMI exchange with 8 peers in every gradient segment, CC4 through 8 ranks, slowest-rank timing,
    fp32 second timing."""
    lines = _bench(["bench.py", "--gpus", "8", "--batch", "4", "--steps", "32", "--warmup", "8"], shared=True,
                   timeout=600)
    assert len(lines) == 1, lines
    out = lines[0]
    assert out["n_gpus"] == 8 and out["allreduce"] == "xgmi" and out["loss_finite"] and out["fp32_loss_finite"]
    assert out["config"]["global_batch"] == 32 and out["config"]["parallelism"] == "dp8"
    assert len(out["per_rank_ms_per_step"]) == 8 and len(out["allreduce_us_per_step"]) == 8
