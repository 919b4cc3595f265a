"""Native engine on a real MI355X: numerics of the HIP kernels vs the plain PyTorch fp32 oracle, end-to-end entry
points, and that the in-tree native library (not an eager fallback) is what runs.

Tolerances are relative L2 errors per tensor:
  independent forwards (ReLU / max-pool mask flips at |z|~0 dominate): fp32 <= 1e-2, bf16 <= 5e-2 per tensor;
  flip-aware (the oracle forced onto the engine's forward): fp32 (3xbf16 MFMA) <= 1e-4, bf16 <= 3e-3;
  8-step trajectory, whole parameter vector: fp32 <= 1e-4, bf16 <= 3e-2.
"""
import json
import os
import subprocess
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "bench"))

pytestmark = pytest.mark.gpu


def _loaded_native_libs():
    with open("/proc/self/maps") as f:
        return {line.split()[-1] for line in f if "libdca_engine" in line}


def test_native_library_loaded_in_tree(gpu):
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    data, labels = synthetic_cifar(64)
    eng = NetResDeepEngine(NetResDeep().to(gpu), data.to(gpu), labels.to(gpu), EngineConfig())
    eng.close()
    libs = _loaded_native_libs()
    assert libs and all(p.startswith(ROOT) for p in libs), libs


@pytest.mark.parametrize("dtype,persistent,B,graph", [
    ("fp32", True, 32, True),   # image-sliced persistent kernel, fp32-accurate (3xbf16) MFMA
    ("bf16", True, 32, True),
    ("bf16", True, 32, False),
    ("bf16", True, 16, True),   # ragged last batch of an epoch
    ("fp32", True, 20, True),
    ("fp32", True, 64, True),   # main_no_ddp.py's batch
    ("fp32", False, 32, True),  # multi-kernel engine (exact fp32 MFMA)
    ("bf16", False, 32, True),
])
def test_one_step_matches_oracle(gpu, dtype, persistent, B, graph):
    """Independent forwards: ReLU / max-pool masks may flip where a pre-activation is ~0, so the backward is
    compared in relative L2 at a loose bound; the flip-aware test below pins the arithmetic."""
    from engine_diag import compare_one_step
    res = compare_one_step(dtype, 4, B, graph, seed=B, verbose=False, persistent=persistent)
    tol = 1e-2 if dtype == "fp32" else 5e-2
    bad = {k: v for k, v in res.items() if v > tol}
    assert not bad, bad
    assert res["state:resblocks.0.batch_norm.num_batches_tracked"] == 0.0  # nbt += 10 per step
    if dtype == "fp32" and persistent:  # forward activations before any mask can flip: 3xbf16 accuracy
        assert max(res[f"x{i}"] for i in range(10)) < 1e-4 and max(res[f"y{i}"] for i in range(10)) < 1e-4, res


@pytest.mark.parametrize("dtype,B,tol", [("fp32", 32, 1e-4), ("fp32", 20, 1e-4), ("fp32", 64, 1e-4),
                                          ("bf16", 32, 3e-3)])
def test_one_step_flip_aware(gpu, dtype, B, tol):
    """The oracle's forward is forced onto the engine's own conv1 output, stem output and 10 conv outputs
    (straight-through), so BatchNorm statistics, ReLU masks and max-pool argmaxes are the engine's and the
    backward differs by arithmetic only: every activation gradient, every parameter gradient and the updated
    state within `tol` relative L2 (fp32 mode: 3xbf16 products, ~2^-17 each)."""
    from engine_diag import compare_one_step
    res = compare_one_step(dtype, 4, B, True, seed=3 + B, verbose=False, persistent=True, forced=True)
    bad = {k: v for k, v in res.items() if v > tol}
    assert not bad, bad


@pytest.mark.parametrize("dtype,persistent,tol", [("fp32", True, 1e-4), ("bf16", True, 3e-2),
                                                  ("fp32", False, 1e-4)])
def test_trajectory_matches_oracle(gpu, dtype, persistent, tol):
    """8 steps, both sides independent: losses and the whole parameter vector (relative L2) track the fp32
    oracle; the worst single tensor (a bias fed by a few mask flips) within 20x."""
    from engine_diag import trajectory
    tr = trajectory(dtype, 4, 32, 8, persistent=persistent)
    assert tr["param_rel_l2"] < tol and tr["max_param_rel_err"] < 20 * tol, tr
    for le, lr in zip(tr["losses_engine"], tr["losses_ref"]):
        assert abs(le - lr) < 5 * tol * max(1.0, abs(lr)), (le, lr)


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-4), ("bf16", 3e-2)])
def test_trajectory_across_epoch_wrap(gpu, dtype, tol):
    """The device epoch seeded to EPOCH_WRAP - 3: the 8 steps cross the wrap (staging parity, BN partial tags,
    granule tags all continue across it) -- still on the fp32 oracle's trajectory, and bitwise the run from epoch 0
    (same state, same batches: the epoch only names the exchange rounds)."""
    from engine_diag import trajectory
    from distributeddataparallel_cifar10_amd.runtime.engine import EPOCH_WRAP
    plain = trajectory(dtype, 4, 32, 8, persistent=True)
    wrap = trajectory(dtype, 4, 32, 8, persistent=True, seed_epoch=EPOCH_WRAP - 3)
    assert plain["epoch_end"] == 8 and wrap["epoch_end"] == 5, (plain["epoch_end"], wrap["epoch_end"])
    assert wrap["param_rel_l2"] < tol and wrap["max_param_rel_err"] < 20 * tol, wrap
    assert torch.equal(plain["params"], wrap["params"])
    assert plain["losses_engine"] == wrap["losses_engine"]


def test_shared_device_budget_refuses_exact_fill(gpu):
    """One co-residency rule (csrc/engine.hip coresident_budget, mirrored by runtime/engine.py): 8 ranks sharing the
    device at batch_max 8 (8 x 32 live step workgroups = every CU) are refused when the sharing is declared --
    before any step could spin in a BN exchange that cannot complete -- while batch_max 4 is accepted."""
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import (EngineConfig, NetResDeepEngine,
                                                                    max_sliced_batch)
    props = torch.cuda.get_device_properties(gpu)
    assert max_sliced_batch(1, props.multi_processor_count, 8) == (props.multi_processor_count - 1) // 8 // 4
    data, labels = synthetic_cifar(64)
    for bmax, ok in ((8, False), (4, True)):
        eng = NetResDeepEngine(NetResDeep().to(gpu), data.to(gpu), labels.to(gpu), EngineConfig(batch_max=bmax))
        try:
            if ok:
                eng.set_shared_device(8)
            else:
                with pytest.raises(RuntimeError, match="co-residency budget"):
                    eng.set_shared_device(8)
        finally:
            eng.close()


@pytest.mark.parametrize("dtype,tol", [("fp32", 0.03), ("bf16", 0.05)])
def test_learnable_epochs_track_pytorch(gpu, dtype, tol):
    """Three short epochs of learnable synthetic data (label = f(image)) on the sliced engine's ``run_epoch`` -- 20
    full batches + a ragged batch of 16, the reference's epoch mean over len(loader) (main.py:43-44), 10 BN EMAs per
    step, the same order every epoch (no set_epoch) -- against stock PyTorch fp32 (CPU) on the same data.

    This regime is chaotic: at lr 1e-2 the loss spikes while the model fits the class patterns, and a 1e-7 relative
    difference (a different fp32 summation order) grows ~3.5x per step (measured: the engine and the fp32 oracle agree
    to 5 digits for 2 steps, 1e-4 at step 4, 1e-2 by step 8; scratch diagnostics, round 5), so a step-by-step bound
    belongs to the non-learning trajectories (test_trajectory_matches_oracle, 1e-4 over 30 steps).  Here: the first
    epoch's mean within `tol` of the oracle's, both runs learning (third-epoch mean < 0.4 x the first, the loss of a
    uniform guess being 2.30), the third-epoch means within a factor 2.5 of each other, every BN counter exact."""
    import copy
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    from distributeddataparallel_cifar10_amd.utils.oracle import reference_step
    B, n = 32, 32 * 20 + 16
    data, labels = synthetic_cifar(n, seed=3, learnable=True)
    torch.manual_seed(5)
    model = NetResDeep()
    ref = copy.deepcopy(model)
    model = model.to(gpu)
    eng = NetResDeepEngine(model, data.to(gpu), labels.to(gpu), EngineConfig(batch_max=B, dtype=dtype))
    assert eng.kind_name == "sliced"
    nb = (n + B - 1) // B
    eng_means, ref_means = [], []
    for _ in range(3):
        loss_sum, steps = eng.run_epoch(list(range(n)), B)
        assert steps == nb
        eng_means.append(loss_sum / nb)
        tot = 0.0
        for k in range(nb):
            sel = slice(k * B, min((k + 1) * B, n))
            tot += reference_step(ref, data[sel], labels[sel], lr=1e-2, bf16_operands=dtype == "bf16",
                                  fc1_bf16=dtype == "bf16")["loss"]
        ref_means.append(tot / nb)
    eng.close()
    info = (eng_means, ref_means)
    assert abs(eng_means[0] - ref_means[0]) <= tol * ref_means[0], info
    assert eng_means[2] < 0.4 * eng_means[0] and ref_means[2] < 0.4 * ref_means[0], info
    assert eng_means[0] < 2.31 and max(eng_means[2], ref_means[2]) < 2.5 * min(eng_means[2], ref_means[2]), info
    assert all(torch.isfinite(p).all() for p in model.parameters())
    assert int(model.state_dict()["resblocks.0.batch_norm.num_batches_tracked"]) == 10 * 3 * nb


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_prologue_reduction_bitwise(gpu, dtype, monkeypatch):
    """Graph chunks with the prologue reduction (each step's gradient segments applied at the start of the next step's
    launch, one reduction kernel per chunk) train bitwise like one reduction kernel after every step
    (DCA_PKS_PROLOGUE=0): 37 steps = chunks of 16 + 16 + 4 + 1, a ragged batch in between, then the epoch / cursor
    bases and the loss accumulator agree too."""
    import copy
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    data, labels = synthetic_cifar(2048, seed=4, learnable=True)
    torch.manual_seed(9)
    m0 = NetResDeep()
    out = []
    for pro in ("1", "0"):
        monkeypatch.setenv("DCA_PKS_PROLOGUE", pro)
        m = copy.deepcopy(m0).to(gpu)
        eng = NetResDeepEngine(m, data.to(gpu), labels.to(gpu), EngineConfig(batch_max=32, dtype=dtype))
        assert eng.prologue(32) == (pro == "1")  # the prologue form really runs (as resident as the default form)
        eng.set_indices(list(range(2048)))
        eng.set_cursor(0)
        eng.read_loss(reset=True)
        eng.run(32, 36)
        eng.run(20, 1)
        loss, steps = eng.read_loss()
        out.append((loss, steps, eng.epoch(), torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()]),
                    m.resblocks[0].batch_norm.running_var.detach().cpu().clone(),
                    int(m.resblocks[0].batch_norm.num_batches_tracked)))
        eng.close()
    (l1, s1, e1, p1, v1, n1), (l0, s0, e0, p0, v0, n0) = out
    assert s1 == s0 == 37 and e1 == e0 == 37 and n1 == n0 == 370
    assert l1 == l0, (l1, l0)
    assert torch.equal(p1, p0) and torch.equal(v1, v0)


@pytest.mark.parametrize("dtype,tol", [("fp32", 1e-4), ("bf16", 2e-2)])
def test_xgmi_loopback_matches_local(gpu, dtype, tol):
    """The xGMI exchange path at world size 1 with the rank as its own peer (loopback: segment slabs written through
    to the uncached region, flags, peer reads, the averaging SGD -- the reduction kernel's mode-2 form that a
    dedicated multi-GPU node runs) trains like the local path: 3 steps from the same initial state, losses and the
    parameter vector within tolerance (the SGD rounds differently: fma vs multiply-subtract), no exchange error."""
    import copy
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    data, labels = synthetic_cifar(512, seed=8, learnable=True)
    torch.manual_seed(13)
    m0 = NetResDeep()
    out = []
    for loop in (False, True):
        m = copy.deepcopy(m0).to(gpu)
        cfg = EngineConfig(batch_max=32, dtype=dtype, comm="xgmi" if loop else "rccl", loopback=loop)
        eng = NetResDeepEngine(m, data.to(gpu), labels.to(gpu), cfg)
        if loop:
            assert eng.xgmi_selftest()
        eng.set_indices(list(range(512)))
        eng.set_cursor(0)
        eng.read_loss(reset=True)
        eng.run(32, 3)
        loss, steps = eng.read_loss()
        eng.check_errors()  # raises on a set exchange / wait error word
        out.append((loss, steps, torch.cat([p.detach().reshape(-1).cpu() for p in m.parameters()])))
        eng.close()
    (l0, s0, p0), (l1, s1, p1) = out
    assert s0 == s1 == 3 and abs(l0 - l1) <= tol * abs(l0), (l0, l1)
    assert ((p1 - p0).norm() / p0.norm()).item() < tol


def test_graft_smoke(gpu):
    import __graft_entry__
    __graft_entry__.smoke()


def test_flat_ddp_torch_path_on_gpu(gpu):
    """Generic path (FlatBucketDDP + FlatSGD, stock ops) == plain module + torch.optim.SGD on the GPU."""
    import copy
    import torch.nn.functional as F
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD
    torch.manual_seed(0)
    m = NetResDeep().to(gpu)
    ref = copy.deepcopy(m)
    ddp = FlatBucketDDP(m)
    opt = FlatSGD(ddp, lr=1e-2)
    opt_r = torch.optim.SGD(ref.parameters(), lr=1e-2)
    for step in range(3):
        x = torch.randn(8, 3, 32, 32, device=gpu)
        y = torch.randint(0, 10, (8,), device=gpu)
        for model, o in ((ddp, opt), (ref, opt_r)):
            loss = F.cross_entropy(model(x), y)
            o.zero_grad()
            loss.backward()
            o.step()
    for (n, p), q in zip(m.named_parameters(), ref.parameters()):
        assert torch.allclose(p, q, atol=1e-4, rtol=1e-3), n


def _run(args, timeout=600):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    return subprocess.run([sys.executable] + args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)


def test_main_single_gpu(gpu, tmp_path):
    ck = tmp_path / "birds_vs_airplanes.pt"
    r = _run(["main.py", "--synthetic", "4096", "--epochs", "1", "--max-steps", "20", "--checkpoint-path", str(ck),
              "--port", "29561"])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Training loss" in r.stdout and "training time:" in r.stdout
    sd = torch.load(str(ck), weights_only=True)
    assert len(sd) == 66 and int(sd["resblocks.0.batch_norm.num_batches_tracked"]) == 200


@pytest.mark.parametrize("batch", [64, 96])
def test_main_no_ddp_batches(gpu, batch):
    """main_no_ddp.py on its dedicated GPU: batch 64 (the reference's) runs on the sliced engine over the full
    device through the automatic choice (no explicit persistent=True, so a device or batch that does not fit falls
    back instead of raising); batch 96 (above the fused engine's 64) runs on the ops-layer kernels."""
    r = _run(["main_no_ddp.py", "--synthetic", "2048", "--epochs", "1", "--max-steps", "12", "--batch-size",
              str(batch)])
    assert r.returncode == 0, r.stderr[-3000:]
    assert "Epoch 1, Training loss" in r.stdout and "training time:" in r.stdout, r.stdout[-2000:]


def test_full_device_engine_choice(gpu):
    """FusedDDPTrainer(full_device=True) at batch 64: the automatic choice takes the sliced engine on all CUs."""
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
    data, labels = synthetic_cifar(256, seed=2)
    tr = FusedDDPTrainer(NetResDeep().to(gpu), data.to(gpu), labels.to(gpu), batch_max=64, full_device=True)
    try:
        assert tr.engine.kind_name == "sliced"
        tr.engine.set_indices(list(range(256)))
        tr.engine.set_cursor(0)
        tr.engine.read_loss(reset=True)
        tr.engine.run(64, 2)
        loss, steps = tr.engine.read_loss()
        assert steps == 2 and loss == loss
    finally:
        tr.close()


def test_bench_contract(gpu):
    r = _run(["bench.py", "--steps", "20", "--warmup", "5"])
    assert r.returncode == 0, r.stderr[-3000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec, k
    assert rec["n_gpus"] == 1 and rec["value"] > 0 and rec["loss_finite"]


@pytest.mark.parametrize("persistent", [True, False])
def test_rccl_path_world_size_one(gpu, persistent):
    """comm="rccl" with force_comm at world_size 1: the graph-captured ncclAllReduce (a 1-rank communicator), the
    stream/event wiring and the averaging SGD kernel all run, and give the same training step as the fused-SGD
    world_size-1 engine (an all-reduce over one rank is the identity)."""
    import copy
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    data, labels = synthetic_cifar(256, seed=3)
    torch.manual_seed(11)
    m0 = NetResDeep()
    out = []
    for force in (False, True):
        m = copy.deepcopy(m0).to(gpu)
        eng = NetResDeepEngine(m, data.to(gpu), labels.to(gpu),
                               EngineConfig(batch_max=32, dtype="bf16", persistent=persistent, comm="rccl",
                                            force_comm=force))
        eng.set_indices(list(range(256)))
        eng.set_cursor(0)
        eng.read_loss(reset=True)
        eng.run(32, 5)  # graph replay incl. the captured collective
        loss, steps = eng.read_loss()
        assert steps == 5
        out.append((loss, {k: v.detach().cpu().clone() for k, v in m.state_dict().items()}))
        eng.close()
    (l0, s0), (l1, s1) = out
    # Not bitwise: the fused step rounds p - lr*g as one FMA, the averaging SGD kernel as p - (lr*g)/1, and a
    # last-bit difference in a weight can flip its bf16 operand rounding.  Same step to bf16-operand accuracy.
    assert abs(l0 - l1) <= 1e-4 * abs(l0), (l0, l1)
    for k in s0:
        a, b = s0[k].double(), s1[k].double()
        err = ((a - b).norm() / max(b.norm().item(), 1e-30)).item()
        assert err <= 2e-3, (k, err)


def test_precapture_keeps_graphs_out_of_timed_runs(gpu):
    """precapture() builds both graph chunk sizes; a later run with any step count only replays."""
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
    data, labels = synthetic_cifar(1024, seed=1)
    eng = NetResDeepEngine(NetResDeep().to(gpu), data.to(gpu), labels.to(gpu), EngineConfig(batch_max=32))
    eng.set_indices(list(range(1024)))
    eng.set_cursor(0)
    eng.precapture(32)
    eng.read_loss(reset=True)
    eng.run(32, 21)  # 16 + 5 x 1
    loss, steps = eng.read_loss()
    eng.close()
    assert steps == 21 and loss == loss
