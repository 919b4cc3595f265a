"""Latency of the engine's one-shot xGMI gradient all-reduce (csrc/xgmi_allreduce.hip), one rank per GPU.

    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench/xgmi_allreduce_bench.py
    DCA_BENCH_SHARE_GPU=1 ...   # N ranks sharing GPU 0 (protocol rehearsal: flags, fences, epochs)

Prints one JSON line (rank 0): mean us per all-reduce of the 304 KB NetResDeep gradient, the slowest rank.
"""
import json
import os
import sys


def _mcheck(lib, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib.dca_micro_last_error().decode(errors='replace')}")

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    world, rank = int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("RANK", "0"))
    share = os.environ.get("DCA_BENCH_SHARE_GPU") == "1"
    dev = torch.device("cuda", 0 if share else int(os.environ.get("LOCAL_RANK", "0")))
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo" if share else "nccl", rank=rank, world_size=world,
                            **({} if share else {"device_id": dev}))
    from distributeddataparallel_cifar10_amd.data.synthetic import synthetic_cifar
    from distributeddataparallel_cifar10_amd.models.netresdeep import NetResDeep
    from distributeddataparallel_cifar10_amd.parallel.ddp import FusedDDPTrainer
    data, labels = synthetic_cifar(256, seed=0)
    tr = FusedDDPTrainer(NetResDeep().to(dev), data.to(dev), labels.to(dev), comm="xgmi")
    out = {"n_ranks": world, "shared_gpu": share, "comm": tr.comm}
    if tr.comm == "xgmi":
        tr.engine.xgmi_bench(50)
        us = torch.tensor([tr.engine.xgmi_bench(500)], dtype=torch.float64)
        dist.all_reduce(us, op=dist.ReduceOp.MAX)
        out.update(us_per_allreduce=round(float(us), 2), bytes=76140 * 4)
    if rank == 0:
        print(json.dumps(out), flush=True)
    tr.close()
    dist.destroy_process_group()




def single_process(ws_list=(1, 2, 3), iters=500):
    """Protocol cost with W ranks simulated in ONE process (co-resident kernels on W streams): the lower bound of
    what the all-reduce adds per step, free of the cross-process scheduling of a shared GPU."""
    import ctypes
    from distributeddataparallel_cifar10_amd.runtime import native
    lib = native.load_micro()
    torch.cuda.init()
    for w in ws_list:
        us, err = ctypes.c_float(), ctypes.c_int()
        _mcheck(lib, lib.dca_microbench_xgmi(w, iters, ctypes.byref(us), ctypes.byref(err)), "microbench_xgmi")
        print(json.dumps({"ranks_in_process": w, "us_per_allreduce": round(us.value, 2), "timeout": bool(err.value),
                          "bytes": 76140 * 4}), flush=True)


if __name__ == "__main__":
    if "--single-process" in sys.argv:
        single_process()
    else:
        main()
