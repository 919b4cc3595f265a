"""Data-parallel semantics of the native engine with 2 ranks sharing one MI355X (gloo carries the all-reduce:
RCCL refuses two ranks on one device, so the engine's comm="external" mode lets the host all-reduce the flat
gradient buffer between the two halves of each step).

Checks against a single-process simulation of reference DDP: CC3 init broadcast, CC5 averaged
gradients + SGD, CC4 rank-0 BN buffers at each forward followed by 10 local EMA updates.  Everything except the
RCCL call itself (one ncclAllReduce over the same buffer) is exercised.
"""
import copy
import os
import sys
import traceback

import pytest
import torch
import torch.distributed as dist

from _ranks import spawn_ranks

pytestmark = pytest.mark.gpu
WS, B, STEPS, NDATA = 2, 16, 3, 256


def _simulate(model0, data, labels, order, lr, bf16, fc1_bf16):
    from distributeddataparallel_cifar10_amd.utils.oracle import reference_step
    models = [copy.deepcopy(model0) for _ in range(WS)]
    for s in range(STEPS):
        snap = {k: v.clone() for k, v in models[0].named_buffers()}
        grads = []
        for r in range(WS):
            with torch.no_grad():
                for k, v in models[r].named_buffers():
                    v.copy_(snap[k])
            sel = order[r][s * B:(s + 1) * B]
            out = reference_step(models[r], data[sel], labels[sel], lr=lr, apply_sgd=False, bf16_operands=bf16,
                                 fc1_bf16=fc1_bf16)
            grads.append(out["grads"])
        with torch.no_grad():
            for r in range(WS):
                for n, p in models[r].named_parameters():
                    p -= lr * sum(g[n] for g in grads) / WS
    return models


def _worker(rank, port, dtype, persistent, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=WS)
        from distributeddataparallel_cifar10_amd.data.sampler import distributed_indices
        from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
        from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
        from distributeddataparallel_cifar10_amd.parallel.ddp import broadcast_module_state
        from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine
        dev = torch.device("cuda", 0)
        data, labels = synthetic_cifar(NDATA, seed=5)
        order = [distributed_indices(NDATA, WS, r) for r in range(WS)]
        torch.manual_seed(100 + rank)  # different init per rank; CC3 fixes it
        model = NetResDeep()
        broadcast_module_state(model, 0)  # CC3 (gloo, CPU tensors)
        ref0 = copy.deepcopy(model)
        model = model.to(dev)
        eng = NetResDeepEngine(model, data.to(dev), labels.to(dev),
                               EngineConfig(batch_max=32, dtype=dtype, persistent=persistent, world_size=WS,
                                            rank=rank, comm="external"))
        eng.set_indices(order[rank])
        eng.set_cursor(0)
        eng.read_loss(reset=True)

        def allreduce(t):
            h = t.cpu()
            dist.all_reduce(h)
            t.copy_(h.to(t.device))

        eng.run_external(B, STEPS, allreduce)
        loss, steps = eng.read_loss()
        assert steps == STEPS
        sim = _simulate(ref0, data, labels, order, 1e-2, dtype == "bf16", persistent and dtype == "bf16")[rank]
        tol = 1e-3 if dtype == "fp32" else 3e-2
        sd, rsd = model.state_dict(), sim.state_dict()
        for k in ("fc1.weight", "fc2.bias", "resblocks.0.conv.weight", "resblocks.0.batch_norm.weight",
                  "conv1.weight", "resblocks.0.batch_norm.running_mean", "resblocks.0.batch_norm.running_var"):
            a, b = sd[k].detach().double().cpu(), rsd[k].detach().double()
            err = ((a - b).norm() / b.norm()).item()
            assert err < tol, (k, err)
        assert int(sd["resblocks.0.batch_norm.num_batches_tracked"]) == 10 * STEPS
        # every rank ends with identical parameters
        flat = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
        other = flat.clone()
        dist.broadcast(other, 0)
        assert torch.equal(flat, other)
        eng.close()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("dtype,persistent,kernel", [("bf16", True, "sliced"), ("fp32", True, "sliced"),
                                                     ("fp32", False, "multi"), ("bf16", False, "multi")])
def test_engine_ddp_two_ranks_one_gpu(gpu, port, dtype, persistent, kernel):
    spawn_ranks(_worker, WS, lambda r: (r, port, dtype, persistent))


def _xgmi_worker(rank, ws, port, dtype, persistent, q, comm="xgmi", own_device=False, batch=B, fc_workers=None,
                 prologue=False):
    """One rank of the fused trainer with the one-shot xGMI all-reduce.  By default all ranks share GPU 0: the
    IPC-mapped slabs are then peers on the same device, which exercises the whole protocol -- epochs, parities,
    flags.  own_device=True (tests/test_multigpu.py): rank r on GPU r, so the slabs and flags cross xGMI, and
    comm="rccl" runs the graph-captured RCCL all-reduce instead.  fc_workers: assert whether the sliced step ran
    the fc gradient segments (and their xGMI exchange) on its fc workers.  prologue: the prologue-reduction form
    (DCA_PKS_PROLOGUE=1; each step's segment exchange runs in the next step's launch), all steps in one chunk."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["DCA_XGMI_TIMEOUT_S"] = "30"  # a protocol bug ends as an error flag, not a hang
        if prologue:
            os.environ["DCA_PKS_PROLOGUE"] = "1"
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from distributeddataparallel_cifar10_amd.data.sampler import distributed_indices
        from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
        from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
        from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
        from distributeddataparallel_cifar10_amd.utils.oracle import reference_step
        dev = torch.device("cuda", rank if own_device else 0)
        torch.cuda.set_device(dev)
        data, labels = synthetic_cifar(NDATA, seed=5)
        order = [distributed_indices(NDATA, ws, r) for r in range(ws)]
        torch.manual_seed(100 + rank)
        model = NetResDeep()
        from distributeddataparallel_cifar10_amd.parallel.ddp import broadcast_module_state
        broadcast_module_state(model, 0)
        ref0 = copy.deepcopy(model)
        model = model.to(dev)
        tr = FusedDDPTrainer(model, data.to(dev), labels.to(dev), batch_max=batch, dtype=dtype,
                             persistent=persistent, comm=comm, max_indices=len(order[rank]))
        assert tr.comm == comm, f"asked for {comm}, got {tr.comm} (the xGMI path did not come up?)"
        eng = tr.engine
        if fc_workers is not None:
            assert eng.fc_in_step(batch) == fc_workers, (batch, fc_workers)
        eng.set_indices(order[rank])
        eng.set_cursor(0)
        eng.read_loss(reset=True)
        import time
        nsteps = STEPS
        if prologue:
            assert eng.prologue(batch), "the prologue form did not engage"
            nsteps = 6
            time.sleep(0.05 * rank)  # uneven start; the steps' exchanges then pace each other
            eng.run(batch, nsteps)  # one graph chunk: steps 2.. reduce the previous step in their prologue
            eng.sync()
        else:
            for s in range(STEPS):  # uneven producer timing: ranks reach each step's all-reduce at different times
                time.sleep(0.03 * ((rank + s) % ws))
                eng.run(batch, 1)  # graph-captured step, the all-reduce inside the graph
                eng.sync()
                print(f"[rank {rank}/{ws}] step {s} done", file=sys.stderr, flush=True)
        loss, steps = eng.read_loss()
        assert steps == nsteps
        _check_vs_simulation(model, ref0, data, labels, order, rank, ws, nsteps, batch, dtype, persistent)
        tr.close()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _simulate_ddp(ref0, data, labels, order, ws, steps, batch, dtype, persistent):
    """Single-process simulation of reference DDP over `ws` ranks (CC4 rank-0 buffers, CC5 averaged gradients)."""
    from distributeddataparallel_cifar10_amd.utils.oracle import reference_step
    models = [copy.deepcopy(ref0) for _ in range(ws)]
    for s in range(steps):
        snap = {k: v.clone() for k, v in models[0].named_buffers()}
        grads = []
        for r in range(ws):
            with torch.no_grad():
                for k, v in models[r].named_buffers():
                    v.copy_(snap[k])
            sel = order[r][s * batch:(s + 1) * batch]
            out = reference_step(models[r], data[sel], labels[sel], lr=1e-2, apply_sgd=False,
                                 bf16_operands=dtype == "bf16", fc1_bf16=persistent and dtype == "bf16")
            grads.append(out["grads"])
        with torch.no_grad():
            for r in range(ws):
                for n, p in models[r].named_parameters():
                    p -= 1e-2 * sum(g[n] for g in grads) / ws
    return models


def _check_vs_simulation(model, ref0, data, labels, order, rank, ws, steps, batch, dtype, persistent):
    """This rank's state tracks the DDP simulation; parameters are bitwise identical on every rank."""
    sim = _simulate_ddp(ref0, data, labels, order, ws, steps, batch, dtype, persistent)[rank]
    tol = 1e-3 if dtype == "fp32" else 3e-2
    sd, rsd = model.state_dict(), sim.state_dict()
    for k in ("fc1.weight", "fc2.bias", "resblocks.0.conv.weight", "resblocks.0.batch_norm.weight",
              "conv1.weight", "resblocks.0.batch_norm.running_mean", "resblocks.0.batch_norm.running_var"):
        a, b = sd[k].detach().double().cpu(), rsd[k].detach().double()
        err = ((a - b).norm() / b.norm()).item()
        assert err < tol, (k, err)
    # bitwise-identical parameters on every rank (fixed rank-order summation)
    flat = torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()])
    other = flat.clone()
    dist.broadcast(other, 0)
    assert torch.equal(flat, other)


def _wrap_worker(rank, ws, port, dtype, q):
    """Two runs from the same state over the same batches, the second with the device epoch seeded to EPOCH_WRAP - 3
    and every xGMI exchange flag to 2^32 - 3, so its 8 steps cross both wraps: bitwise the first run's parameters,
    and on the DDP simulation's trajectory."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["DCA_XGMI_TIMEOUT_S"] = "30"
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from distributeddataparallel_cifar10_amd.data.sampler import distributed_indices
        from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
        from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
        from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer, broadcast_module_state
        from distributeddataparallel_cifar10_amd.runtime.engine import EPOCH_WRAP
        dev = torch.device("cuda", 0)
        torch.cuda.set_device(dev)
        batch, steps = 8, 8
        data, labels = synthetic_cifar(NDATA, seed=7)
        order = [distributed_indices(NDATA, ws, r) for r in range(ws)]
        torch.manual_seed(200 + rank)
        ref0 = NetResDeep()
        broadcast_module_state(ref0, 0)
        finals = []
        for seeded in (False, True):
            model = copy.deepcopy(ref0).to(dev)
            tr = FusedDDPTrainer(model, data.to(dev), labels.to(dev), batch_max=batch, dtype=dtype, comm="xgmi",
                                 max_indices=len(order[rank]))
            assert tr.comm == "xgmi"
            eng = tr.engine
            if seeded:
                dist.barrier()  # no rank steps while the flags are seeded (peers write into each other's flags)
                eng.set_epoch(EPOCH_WRAP - 3, 2 ** 32 - 3)
                dist.barrier()
            eng.set_indices(order[rank])
            eng.set_cursor(0)
            eng.read_loss(reset=True)
            eng.run(batch, steps)
            _, n = eng.read_loss()  # raises on any exchange timeout
            assert n == steps
            if seeded:
                assert eng.epoch() == 5, eng.epoch()
                _check_vs_simulation(model, ref0, data, labels, order, rank, ws, steps, batch, dtype, True)
            finals.append(torch.cat([p.detach().reshape(-1).cpu() for p in model.parameters()]))
            tr.close()
        assert torch.equal(finals[0], finals[1])
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_xgmi_epoch_wrap_two_ranks_one_gpu(gpu, port, dtype):
    spawn_ranks(_wrap_worker, 2, lambda r: (r, 2, port, dtype))


@pytest.mark.parametrize("ws,dtype,persistent,batch", [(2, "bf16", True, B), (4, "bf16", True, 12),
                                                       (2, "fp32", True, B), (2, "fp32", False, B),
                                                       (3, "fp32", True, 8), (4, "fp32", True, 8),
                                                       (8, "bf16", True, 4), (8, "fp32", True, 4),
                                                       (8, "bf16", False, 4)])
def test_xgmi_allreduce_ranks_one_gpu(gpu, port, ws, dtype, persistent, batch):
    """ws=8 (the node's world size): the sliced engine's reduction exchange with 8 peers (rank_sum_n<8> in
    seg_exchange), its fc-worker exchange with 8 peers (construction self-test, FusedDDPTrainer), CC4 through 8
    ranks, the multi-kernel engine's k_xgmi_ar_sgd with 8 peers.  A per-rank batch of 4 keeps each rank's step
    grid (16 workgroups, one CU each) at half its 256 / 8 CU budget (batch 8 fills it exactly: no slack while a
    peer's kernels still hold CUs), and every rank has one hardware queue
    (tests/_ranks.py: with the default 4 per process, 8 processes oversubscribed the hardware scheduler)."""
    spawn_ranks(_xgmi_worker, ws, lambda r: (r, ws, port, dtype, persistent), dict(batch=batch))


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_xgmi_fc_workers_two_ranks_one_gpu(gpu, port, dtype):
    """Batch 8 on 2 ranks sharing the GPU: both steps with their fc workers (2 x 97 workgroups) and a peer's
    reduction fit on the device together, so the fc workers' in-step xGMI exchange runs (the path of the
    cross-device runs) and must match the DDP simulation bitwise-consistently on both ranks."""
    spawn_ranks(_xgmi_worker, 2, lambda r: (r, 2, port, dtype, True), dict(batch=8, fc_workers=True))


@pytest.mark.parametrize("dtype", ["bf16", "fp32"])
def test_xgmi_prologue_two_ranks_one_gpu(gpu, port, dtype):
    """The prologue-reduction form with the xGMI exchange (2 ranks sharing the GPU, batch 8): each step's segment
    exchange and SGD run at the start of the next step's launch, whose step workgroups wait for them under the
    exchange deadline.  Must track the DDP simulation with bitwise-equal parameters on both ranks."""
    spawn_ranks(_xgmi_worker, 2, lambda r: (r, 2, port, dtype, True), dict(batch=8, prologue=True))


def test_bench_two_ranks_shared_gpu(gpu, port):
    """The driver's multi-GPU bench command (torch.distributed.run, one rank per GPU) rehearsed with 2 ranks on
    this box's one GPU: JSON contract, whole-job value, the xGMI all-reduce actually in use.  The launcher's
    environment has no HSA_ENABLE_IPC_MODE_LEGACY: bench.py must select the dmabuf IPC mode itself (the xGMI
    all-reduce maps the peers' regions through IPC handles)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DCA_BENCH_SHARE_GPU="1", DCA_XGMI_TIMEOUT_S="60")
    env.pop("HSA_ENABLE_IPC_MODE_LEGACY", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2", "--master-addr",
           "127.0.0.1", "--master-port", str(port), "bench.py", "--gpus", "2", "--batch", "16", "--steps", "48",
           "--warmup", "16"]  # (2 x batch 32 would fill the device exactly: refused by the co-residency rule)
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["n_gpus"] == 2 and out["steps"] == 48 and out["allreduce"] == "xgmi" and out["loss_finite"]
    assert out["config"]["global_batch"] == 32 and out["config"]["parallelism"] == "dp2"
    assert out["value"] > 0


def test_bench_self_launch_sweep_shared_gpu(gpu):
    """``python bench.py --sweep 1,2`` (no torchrun): bench.py spawns each rank group itself (reference
    main.py:84 mp.spawn), rank 0 prints the per-N JSON line (whole-job value, per-rank step times, the xGMI
    all-reduce time per step) and the parent prints the scaling summary.  Rehearsed with the ranks sharing this
    box's one GPU (DCA_BENCH_SHARE_GPU=1)."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, DCA_BENCH_SHARE_GPU="1", DCA_XGMI_TIMEOUT_S="60")
    env.pop("WORLD_SIZE", None)
    cmd = [sys.executable, "bench.py", "--sweep", "1,2", "--batch", "16", "--steps", "48", "--warmup", "16"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=400)
    assert r.returncode == 0, r.stderr[-4000:]
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 3, r.stdout
    one, two, summary = recs
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2 and two["allreduce"] == "xgmi" and two["loss_finite"]
    assert len(two["per_rank_ms_per_step"]) == 2 and all(v > 0 for v in two["allreduce_us_per_step"])
    assert set(summary["scaling_efficiency"]) == {"1", "2"} and summary["scaling_efficiency"]["1"] == 1.0


def _stall_worker(rank, ws, port, q):
    """Rank 1 stops after 3 steps (fault injection: a peer that stops stepping); rank 0's run_epoch must raise
    within 16 steps of the stall, not at the epoch end (the error words are checked after every 8-step chunk and the
    exchanges fail fast once one has timed out)."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["DCA_XGMI_TIMEOUT_S"] = "1"
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
        from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
        from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
        dev = torch.device("cuda", 0)
        data, labels = synthetic_cifar(NDATA, seed=5)
        torch.manual_seed(0)
        tr = FusedDDPTrainer(NetResDeep().to(dev), data.to(dev), labels.to(dev), batch_max=8, dtype="bf16",
                             comm="xgmi", max_indices=NDATA)
        assert tr.comm == "xgmi"
        eng = tr.engine
        batch, good = 8, 3
        if rank == 0:
            raised = False
            try:
                eng.run_epoch(list(range(NDATA)), batch)  # 32 steps; the peer is gone after step 3
            except RuntimeError as ex:
                raised = "xGMI" in str(ex)
            assert raised, "a peer that stopped stepping was not reported"
            _, steps = eng.read_loss()
            assert good < steps <= good + 16, steps
        else:
            eng.set_indices(list(range(NDATA)))
            eng.set_cursor(0)
            eng.run(batch, good)
            eng.sync()
        dist.barrier()
        tr.close()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_peer_stall_raises_within_16_steps(gpu, port):
    spawn_ranks(_stall_worker, 2, lambda r: (r, 2, port))


def _slow_peer_worker(rank, ws, port, q):
    """Rank 1 pauses 3 s (> the 1 s exchange deadline) after 3 steps, then keeps stepping.  Rank 0's wait expires; from
    then on rank 0 neither publishes nor waits, so rank 1's next exchanges expire too: BOTH ranks must report the
    error (before round 5 rank 0 kept publishing ahead and the slow rank passed its waits on later epochs' slabs,
    silently summing mixed epochs)."""
    try:
        import time
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        os.environ["DCA_XGMI_TIMEOUT_S"] = "1"
        dist.init_process_group("gloo", rank=rank, world_size=ws)
        from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
        from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
        from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
        dev = torch.device("cuda", 0)
        data, labels = synthetic_cifar(NDATA, seed=5)
        torch.manual_seed(0)
        tr = FusedDDPTrainer(NetResDeep().to(dev), data.to(dev), labels.to(dev), batch_max=8, dtype="bf16",
                             comm="xgmi", max_indices=NDATA)
        assert tr.comm == "xgmi"
        eng = tr.engine
        batch, good = 8, 3
        eng.set_indices(list(range(NDATA)))
        eng.set_cursor(0)
        eng.read_loss(reset=True)
        raised = False
        try:
            if rank == 1:
                eng.run(batch, good)
                eng.sync()
                time.sleep(3.0)
                eng.run_checked(batch, NDATA // batch - good)
            else:
                eng.run_checked(batch, NDATA // batch)
        except RuntimeError as ex:
            raised = "xGMI" in str(ex)
        assert raised, f"rank {rank} did not report the expired exchange"
        dist.barrier()
        tr.close()
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_slow_peer_every_rank_reports(gpu, port):
    spawn_ranks(_slow_peer_worker, 2, lambda r: (r, 2, port))
