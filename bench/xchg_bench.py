"""Calibrate the in-kernel all-gather (BN-statistics exchange) of a persistent design on the GPU."""
import ctypes
import json
import os
import sys


def _mcheck(lib, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib.dca_micro_last_error().decode(errors='replace')}")

import torch  # noqa: F401

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.runtime import native  # noqa: E402

lib = native.load_micro()
for G in (8, 16, 32, 64, 128):
    for nth in (1024, 256):
        for sleep in (2,):
            res = {}
            for rounds in (0, 20):
                us, err = ctypes.c_float(), ctypes.c_int()
                _mcheck(lib, lib.dca_microbench_xchg(G, nth, rounds, 20, sleep, ctypes.byref(us), ctypes.byref(err)),
                             "xchg")
                res[rounds] = (us.value, err.value)
            per = (res[20][0] - res[0][0]) / 20
            print(json.dumps({"G": G, "threads": nth, "sleep": sleep, "launch_us": round(res[0][0], 2),
                              "per_round_us": round(per, 3), "timeouts": res[20][1]}), flush=True)
