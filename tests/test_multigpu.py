"""Cross-device data parallelism: one rank per GPU on a multi-GPU MI355X node (skipped below 2 devices, so the
1-GPU tier collects and skips them; on an 8-GPU node they run unchanged).

* the fused trainer's DDP step against the single-process oracle simulation with the slabs / flags crossing xGMI
  (comm="xgmi") and with the graph-captured RCCL all-reduce (comm="rccl"); bitwise-equal parameters on all ranks;
* the driver's own bench command (torch.distributed.run, one rank per GPU) with both all-reduce paths.
"""
import json
import os
import subprocess
import sys

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = [pytest.mark.gpu, pytest.mark.multigpu]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _ngpu() -> int:
    return torch.cuda.device_count()


needs2 = pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per device)")


@needs2
@pytest.mark.parametrize("comm", ["xgmi", "rccl"])
def test_ddp_engine_cross_device(gpu, port, comm):
    from test_ddp_engine_gpu import _xgmi_worker
    ws = min(_ngpu(), 8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_xgmi_worker, args=(r, ws, port, "bf16", True, q, comm, True)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=600) for _ in procs]
    for p in procs:
        p.join(timeout=120)
    bad = [r for r in res if r[1]]
    assert not bad, "\n".join(f"rank {r}:\n{e}" for r, e in bad)


@needs2
@pytest.mark.parametrize("allreduce", ["xgmi", "rccl"])
def test_bench_one_rank_per_gpu(gpu, port, allreduce):
    n = min(_ngpu(), 8)
    env = dict(os.environ, DCA_XGMI_TIMEOUT_S="60")
    env.pop("DCA_BENCH_SHARE_GPU", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(n), "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", str(n), "--steps", "64", "--warmup", "32",
           "--allreduce", allreduce]
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["allreduce"] == allreduce and out["loss_finite"]


@needs2
def test_resnet50_bench_self_launch(gpu):
    """bench/resnet50.py --gpus N spawns one rank per GPU itself (FlatBucketDDP over xGMI, ops kernels); small
    batch / image so it finishes quickly."""
    n = min(_ngpu(), 8)
    cmd = [sys.executable, "bench/resnet50.py", "--gpus", str(n), "--batch", "16", "--image", "64", "--steps", "3",
           "--warmup", "1"]
    r = subprocess.run(cmd, cwd=ROOT, env=dict(os.environ, DCA_XGMI_TIMEOUT_S="60"), capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == n and out["value"] > 0 and out["loss"] == out["loss"]
