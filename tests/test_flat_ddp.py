"""FlatBucketDDP semantics on CPU with gloo, world_size 2 (SURVEY.md section 4 layer 3).

Checks CC3 (init broadcast), CC4 (rank-0 buffers at every forward), CC5 (averaged gradients, bucket-wise,
first bucket launched before the backward ends) and end-to-end equivalence with torch's own DDP.
"""
import copy
import os
import traceback

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD

WS = 2


def _worker(rank, ws, port, fn, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=ws)
    try:
        fn(rank, ws)
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _spawn(fn, port, ws=WS):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, ws, port, fn, q)) for r in range(ws)]
    for p in procs:
        p.start()
    errs = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    bad = [e for e in errs if e[1]]
    assert not bad, "\n".join(f"rank {r}:\n{e}" for r, e in bad)


def _batch(rank, step, n=8):
    g = torch.Generator().manual_seed(1000 * step + rank)
    return torch.randn(n, 3, 32, 32, generator=g), torch.randint(0, 10, (n,), generator=g)


def _case_init_broadcast_and_grad_average(rank, ws):
    torch.manual_seed(100 + rank)  # different init per rank; CC3 must make them equal
    m = NetResDeep()
    ddp = FlatBucketDDP(m, bucket_cap_mb=0.1, first_bucket_mb=0.05)
    assert len(ddp.buckets) >= 2
    # CC3: everyone now holds rank 0's parameters
    ref = [p.detach().clone() for p in m.parameters()]
    for t in ref:
        ts = [torch.empty_like(t) for _ in range(ws)]
        dist.all_gather(ts, t)
        assert all(torch.equal(ts[0], x) for x in ts)
    # CC5: averaged gradients equal the mean of per-rank local gradients
    local = copy.deepcopy(m)
    x, y = _batch(rank, 0)
    F.cross_entropy(local(x), y).backward()
    F.cross_entropy(ddp(x), y).backward()
    for (n, p), lp in zip(m.named_parameters(), local.parameters()):
        g = lp.grad.clone()
        dist.all_reduce(g)
        g /= ws
        assert torch.allclose(p.grad, g, atol=1e-6, rtol=1e-5), n
    # buckets fire in gradient-ready order, the fc bucket first (before conv1's grad exists)
    assert ddp.bucket_fire_order[0] == 0 and sorted(ddp.bucket_fire_order) == list(range(len(ddp.buckets)))


def _case_buffer_broadcast_every_forward(rank, ws):
    torch.manual_seed(7)
    m = NetResDeep()
    ddp = FlatBucketDDP(m)
    bn = m.resblocks[0].batch_norm
    with torch.no_grad():
        bn.running_mean.fill_(float(rank + 1))  # ranks diverge between forwards
    expected = copy.deepcopy(m)
    with torch.no_grad():
        expected.resblocks[0].batch_norm.running_mean.fill_(1.0)  # rank 0's buffer wins (CC4)
    x, _ = _batch(rank, 1)
    with torch.no_grad():
        ddp(x)
        expected(x)  # then 10 local EMA updates on this rank's batch
    assert torch.allclose(bn.running_mean, expected.resblocks[0].batch_norm.running_mean, atol=1e-6)
    assert int(bn.num_batches_tracked) == 10


def _case_flat_buffers_one_broadcast_per_dtype(rank, ws):
    """Buffers are views of one flat tensor per dtype (like the parameters), so CC4 is one in-place broadcast per
    dtype: 2 collectives (fp32 running stats, int64 counters) and no concatenation / copy-back per forward.  The
    ResNet's BN buffers and NetResDeep's shared ResBlock (one BN applied 10x) both stay intact."""
    from distributeddataparallel_cifar10_amd.models.resnet50 import ResNet
    torch.manual_seed(0)
    for m in (NetResDeep(), ResNet([1, 1, 1, 1], num_classes=10)):
        ddp = FlatBucketDDP(m)
        bufs = list(m.buffers())
        flats = {f.dtype: f for f in ddp._flat_buffers}
        assert set(flats) == {torch.float32, torch.int64} and len(ddp._flat_buffers) == 2
        assert sum(f.numel() for f in flats.values()) == sum(b.numel() for b in bufs)
        for b in bufs:  # every buffer lives inside its dtype's flat tensor
            f = flats[b.dtype]
            assert f.data_ptr() <= b.data_ptr() < f.data_ptr() + f.numel() * f.element_size()
        if isinstance(m, NetResDeep):  # the 10 applications still share one BN module
            assert len({id(blk.batch_norm) for blk in m.resblocks}) == 1
        with torch.no_grad():  # ranks diverge between forwards
            for b in bufs:
                b.fill_(rank + 1)
        calls = []
        real = dist.broadcast

        def counting(t, src, group=None, async_op=False):
            calls.append((str(t.dtype), t.numel()))
            return real(t, src, group=group, async_op=async_op)

        dist.broadcast = counting
        try:
            ddp.eval()
            with torch.no_grad():
                ddp(torch.randn(2, 3, 32, 32))  # eval forward: CC4 only, buffers untouched by the BN itself
        finally:
            dist.broadcast = real
        assert sorted(calls) == sorted((str(f.dtype), f.numel()) for f in flats.values()), calls
        assert all(bool((b == 1).all()) for b in bufs)  # rank 0's buffers everywhere
        with torch.profiler.profile(activities=[torch.profiler.ProfilerActivity.CPU]) as prof:
            ddp._broadcast_buffers_now()  # CC4 alone: no cat, no per-buffer copy-back
        ops = [e.name for e in prof.events()]
        assert not [n for n in ops if n in ("aten::copy_", "aten::cat", "aten::_foreach_copy_", "aten::stack")], ops


def _case_matches_torch_ddp(rank, ws):
    torch.manual_seed(3)
    base = NetResDeep()
    a = copy.deepcopy(base)
    b = copy.deepcopy(base)
    ours = FlatBucketDDP(a, bucket_cap_mb=0.1)
    opt_a = FlatSGD(ours, lr=1e-2)
    theirs = torch.nn.parallel.DistributedDataParallel(b)
    opt_b = torch.optim.SGD(b.parameters(), lr=1e-2)
    for step in range(3):
        x, y = _batch(rank, step)
        for model, opt in ((ours, opt_a), (theirs, opt_b)):
            loss = F.cross_entropy(model(x), y)
            opt.zero_grad()
            loss.backward()
            opt.step()
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        assert torch.allclose(pa, pb, atol=1e-5, rtol=1e-4), n
    sa, sb = a.state_dict(), b.state_dict()
    for k in sa:
        if sa[k].dtype.is_floating_point:
            assert torch.allclose(sa[k], sb[k], atol=1e-5, rtol=1e-4), k
        else:
            assert torch.equal(sa[k], sb[k]), k


@pytest.mark.parametrize("case", [_case_init_broadcast_and_grad_average, _case_buffer_broadcast_every_forward,
                                  _case_matches_torch_ddp, _case_flat_buffers_one_broadcast_per_dtype])
def test_flat_ddp_gloo(case, port):
    _spawn(case, port)


def test_flat_ddp_single_process_zero_grad_none():
    m = NetResDeep()
    ddp = FlatBucketDDP(m)
    opt = torch.optim.SGD(m.parameters(), lr=0.1)
    x, y = _batch(0, 0)
    F.cross_entropy(ddp(x), y).backward()
    g1 = ddp.flat_grad.clone()
    opt.zero_grad(set_to_none=True)  # drops the views; the hook must fold grads back in
    F.cross_entropy(ddp(x), y).backward()
    assert all(p.grad.data_ptr() >= ddp.flat_grad.data_ptr() for p in m.parameters())
    assert torch.allclose(ddp.flat_grad, g1, atol=1e-6)


def _fused_sgd_worker(rank, ws, port, q):
    import traceback
    try:
        import os
        import torch.distributed as dist
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        if ws > 1:
            dist.init_process_group("gloo", rank=rank, world_size=ws)
        import torch.nn as nn
        from distributeddataparallel_cifar10_amd.parallel.flat_ddp import FlatBucketDDP, FlatSGD
        torch.manual_seed(0)
        a = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.Flatten(), nn.Linear(8 * 8 * 8, 10))
        b = nn.Sequential(nn.Conv2d(3, 8, 3, padding=1), nn.ReLU(), nn.Flatten(), nn.Linear(8 * 8 * 8, 10))
        b.load_state_dict(a.state_dict())
        da = FlatBucketDDP(a, bucket_cap_mb=0.005, first_bucket_mb=0.002)
        db = FlatBucketDDP(b, bucket_cap_mb=0.005, first_bucket_mb=0.002)
        assert len(da.buckets) >= 2
        oa = FlatSGD(da, lr=0.05, momentum=0.9, weight_decay=1e-3)
        ob = FlatSGD(db, lr=0.05, momentum=0.9, weight_decay=1e-3, overlap=True)
        for step in range(4):
            g = torch.Generator().manual_seed(10 * step + rank)
            x, y = torch.randn(4, 3, 8, 8, generator=g), torch.randint(0, 10, (4,), generator=g)
            for d, o in ((da, oa), (db, ob)):
                o.zero_grad()
                nn.functional.cross_entropy(d(x), y).backward()
                o.step()
            torch.testing.assert_close(db.flat, da.flat, rtol=1e-6, atol=1e-7, msg=f"step {step}")
        q.put((rank, None))
    except Exception:
        q.put((rank, traceback.format_exc()))


@pytest.mark.parametrize("ws", [1, 2])
def test_fused_overlapped_sgd_matches_step(ws):
    """FlatSGD(overlap=True): per-bucket updates issued during the backward (behind each bucket's all-reduce)
    give the same parameters as one SGD step after the backward (momentum + weight decay, 4 steps)."""
    import torch.multiprocessing as mp
    port = 29600 + ws
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_fused_sgd_worker, args=(r, ws, port, q)) for r in range(ws)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    bad = [r for r in res if r[1]]
    assert not bad, "\n".join(f"rank {r}:\n{e}" for r, e in bad)


def test_xgmi_crossover_pick():
    """XgmiComm.calibrate's decision rule (CPU): two-shot from the smallest size where it wins at that size and
    every larger one; an isolated small-size win is noise; no win means one-shot everywhere."""
    from distributeddataparallel_cifar10_amd.parallel.xgmi import XgmiComm
    sizes = [1 << 16, 1 << 18, 1 << 20, 1 << 22]
    pick = XgmiComm.pick_crossover
    assert pick(sizes, [10, 20, 40, 80], [12, 18, 30, 50]) == 1 << 18
    assert pick(sizes, [10, 20, 40, 80], [9, 25, 30, 50]) == 1 << 20   # the 64 KiB win is not a crossover
    assert pick(sizes, [10, 20, 40, 80], [11, 21, 41, 81]) is None
    assert pick(sizes, [10, 20, 40, 80], [9, 19, 39, 79]) == 1 << 16
    assert pick(sizes, [10, 20, 40, 80], [9, 19, 39, 81]) is None       # loses at the largest size
