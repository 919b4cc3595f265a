"""Calibrate BN-statistics exchange variants of the sliced engine (bench/micro/engine_micro.hip k_mb_bnx).

Per round every workgroup "computes" for work + hash % jitter (10-ns ticks), publishes 64 fp32 partials and waits
for the 64 sums over all G workgroups.  per_round_us = (T(40 rounds) - T(0)) / 40 - the mean emulated work, i.e.
the exchange cost including the wait for the slowest publisher.  Variants: see k_mb_bnx."""
import ctypes
import json
import os
import sys

import torch  # noqa: F401  (loads the HIP runtime first)

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from distributeddataparallel_cifar10_amd.runtime import native  # noqa: E402

NAMES = {0: "1hop-8B", 1: "1hop-4B-selftag", 2: "2hop-8B", 3: "2hop-4B-selftag", 4: "2hop-xcc-census-L2"}


def run(lib, v, G, rounds, work, jitter, iters=5):
    us, err = ctypes.c_float(), ctypes.c_int()
    rc = lib.dca_microbench_bnx(v, G, rounds, work, jitter, iters, ctypes.byref(us), ctypes.byref(err))
    if rc != 0:
        raise RuntimeError(lib.dca_micro_last_error().decode(errors="replace"))
    return us.value, err.value


def main():
    lib = native.load_micro()
    Gs = [int(x) for x in (sys.argv[1] if len(sys.argv) > 1 else "32,64,128,256").split(",")]
    global VARIANTS
    VARIANTS = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "0,1,2,3,4").split(",")]
    for work, jitter in ((150, 0), (150, 100)):
        for G in Gs:
            for v in VARIANTS:
                t0, e0 = run(lib, v, G, 0, work, jitter)
                t1, e1 = run(lib, v, G, 40, work, jitter)
                mean_work_us = (work + (jitter - 1) / 2.0 if jitter else work) / 100.0
                print(json.dumps({"variant": NAMES[v], "G": G, "work_us": work / 100.0, "jitter_us": jitter / 100.0,
                                  "per_round_us": round((t1 - t0) / 40 - mean_work_us, 3),
                                  "timeouts": e0 | e1}), flush=True)


if __name__ == "__main__":
    main()
