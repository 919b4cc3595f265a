"""Multi-process helpers of the GPU tests: spawn N rank processes, collect their results, and make sure none of them
outlives its test.

Ranks that share one GPU (the shared-GPU rehearsals of the multi-GPU paths) each get ONE hardware queue
(``GPU_MAX_HW_QUEUES=1``, inherited at spawn): with 8 processes of up to 4 queues each the device's hardware
scheduler is oversubscribed and time-slices the queues, which stalls the ranks' spinning exchange kernels for whole
time slices (and once ended in an illegal-instruction queue abort in two processes at start-up).  One queue per
rank keeps all of them mapped.  A rank process still alive after the join timeout is killed (its own PID), so a
stuck rank cannot keep holding CUs that the next test's grids need.
"""
from __future__ import annotations

import os
import time

import torch.multiprocessing as mp


_LAST_GROUP: list = []  # mp.Process objects of the previous rank group (this test process spawned them)


def _previous_group_gone(wait_s: float = 60.0) -> None:
    """No process of the previous rank group may still exist when the next one starts: its hardware queues and IPC
    mappings would overlap the new group's start-up (round 4's illegal-instruction abort hit two ranks' first stock
    kernels while the previous 8-rank group was still being torn down -- docs/STATUS.md).  Waits, then kills.  Works
    on the Process objects, never on bare PIDs: once a process has been reaped its PID may belong to someone else,
    and Process.is_alive() / kill() never signal a reaped child."""
    deadline = time.time() + wait_s
    for p in _LAST_GROUP:
        p.join(timeout=max(0.0, deadline - time.time()))
        if p.is_alive():
            p.kill()
            p.join(timeout=30)
    _LAST_GROUP.clear()


def spawn_ranks(target, ws: int, args_for_rank, kwargs=None, shared: bool = True, timeout: float = 600.0):
    """Run ``target(*args_for_rank(r), q, **kwargs)`` in ws spawned processes; every rank puts (rank, error-or-None)
    on q.  Raises AssertionError with the failing ranks' tracebacks."""
    _previous_group_gone()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    saved = os.environ.get("GPU_MAX_HW_QUEUES")
    if shared and ws > 1:
        os.environ["GPU_MAX_HW_QUEUES"] = "1"
    try:
        procs = [ctx.Process(target=target, args=(*args_for_rank(r), q), kwargs=kwargs or {}) for r in range(ws)]
        for p in procs:
            p.start()
            _LAST_GROUP.append(p)
    finally:
        if saved is None:
            os.environ.pop("GPU_MAX_HW_QUEUES", None)
        else:
            os.environ["GPU_MAX_HW_QUEUES"] = saved
    try:
        res = [q.get(timeout=timeout) for _ in procs]
    finally:
        for p in procs:
            p.join(timeout=60)
        for p in procs:
            if p.is_alive():
                p.kill()
                p.join(timeout=30)
    bad = [r for r in res if r[1]]
    assert not bad, "\n".join(f"rank {r}:\n{e}" for r, e in bad)
