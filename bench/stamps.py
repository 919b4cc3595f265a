"""Where does a training step spend its time?  (diagnostic; needs the stamps build)

Runs the engine built with -DDCA_STAMPS (in-kernel s_memtime/s_memrealtime at phase boundaries) and prints, per
kernel of one step: dispatch skew across workgroups, per-phase medians (shader cycles), kernel span, and the
gap to the previous kernel (last workgroup end -> first workgroup start, 100 MHz realtime clock).
Also calibrates the launch floor with graphs of empty / load-only kernels (dca_microbench).

    DCA_ENGINE_VARIANT=stamps python bench/stamps.py
"""
from __future__ import annotations


def _mcheck(lib, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed: {lib.dca_micro_last_error().decode(errors='replace')}")

import ctypes
import json
import os
import sys

os.environ.setdefault("DCA_ENGINE_VARIANT", "stamps")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model.resnet import NetResDeep  # noqa: E402
from distributeddataparallel_cifar10_amd.runtime import native  # noqa: E402
from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine  # noqa: E402

SLOTS = ["stem+conv0"] + [f"fwd{i}" for i in range(1, 10)] + ["head1", "head2"] + \
        [f"bwd{i}" for i in range(9, -1, -1)] + ["reduce"]


def microbench(lib):
    out = {}
    kinds = ((0, "empty"), (1, "shared32K_serialreduce"), (2, "1float_private"), (3, "private32K"),
             (4, "fresh32K_sameWG"), (5, "fresh32K_nextWG"), (6, "fresh32K_broadcast"))
    for kind, name in kinds:
        for grid in (128, 256):
            us = ctypes.c_float()
            _mcheck(lib, lib.dca_microbench(kind, 23, grid, 200, ctypes.byref(us)), "microbench")
            out[f"{name}/grid{grid}"] = round(us.value, 3)
    return out


# persistent-kernel stamp ids (netresdeep_persistent.hip PK_STAMP): 0 start, 1 stem end, 2+i fwd block i conv end,
# 12 bn9 stats, 13 head end, 14+k bwd block 9-k end, 24 kernel end, 25/26 and 27/28 around the block-5 exchanges,
# 29 stem staged, 30 stem MFMA done, 31 head pooled, 32 fc1 done, 33 CE done, 34 stem-bwd staged, 35 stem-bwd MFMA,
# block detail: 36 bwd5 published, 38 bwd5 wgrad(6) done, 37 bwd5 dy staged, 39 fwd6 apply done
PK_INTERVALS = ([("stem", 0, 1), ("stem.stage", 0, 29), ("stem.mfma", 29, 30), ("stem.tail", 30, 1)] +
                [(f"fwd{i}", 1 + i, 2 + i) for i in range(10)] +
                [("bn9+head_start", 11, 12), ("head", 12, 13), ("head.pool", 12, 31), ("head.fc1", 31, 32),
                 ("head.ce", 32, 33), ("head.dp", 33, 13)] +
                [(f"bwd{9 - k}", 13 + k, 14 + k) for k in range(10)] +
                [("stem_bwd", 23, 24), ("stem_bwd.stage", 23, 34), ("stem_bwd.mfma", 34, 35),
                 ("stem_bwd.tail", 35, 24),
                 ("fwd5_pre_xchg", 7, 25), ("fwd5_xchg", 25, 26), ("fwd6_apply", 26, 39), ("fwd6_conv", 39, 8),
                 ("head.ce.hh", 32, 40), ("head.ce.logits", 40, 41), ("head.ce.softmax_dh", 41, 42),
                 ("head.ce.rest", 42, 33), ("stem.bfrag", 29, 43), ("stem.iter0", 43, 44), ("stem.iter1-3", 44, 30),
                 ("bwd5.dz+csum+pub", 17, 36), ("bwd5.wgrad6", 36, 38), ("bwd5.xT", 38, 27), ("bwd5_wait", 27, 28),
                 ("bwd5.dy", 28, 37), ("bwd5.dgrad", 37, 18)])


def persistent_report(st):
    """Per-phase durations of the persistent kernel (median over workgroups, shader cycles and us)."""
    flat = st[24:32].transpose(1, 0, 2, 3).reshape(256, 64, 2)  # [wg][stamp][memtime|realtime]
    valid = flat[:, 0, 1] != 0
    f = flat[valid].astype(np.int64)
    out = []
    for name, a, b in PK_INTERVALS:
        cyc = np.median(f[:, b, 0] - f[:, a, 0])
        us = np.median(f[:, b, 1] - f[:, a, 1]) / 100.0
        out.append({"phase": name, "cyc": int(cyc), "us": round(float(us), 2)})
    tot = np.median(f[:, 24, 1] - f[:, 0, 1]) / 100.0
    return out, round(float(tot), 2)


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    if len(sys.argv) > 2 and sys.argv[2] == "persistent":
        dev = torch.device("cuda", 0)
        data = torch.randint(0, 256, (4096, 3, 32, 32), dtype=torch.uint8, device=dev)
        labels = torch.randint(0, 10, (4096,), device=dev)
        model = NetResDeep().to(dev)
        eng = NetResDeepEngine(model, data, labels, EngineConfig(batch_max=32, dtype="bf16", persistent=True))
        eng.set_indices(np.arange(4096, dtype=np.int32))
        eng.set_cursor(0)
        eng.run(32, 50)
        eng.sync()
        eng.run(32, 1)
        eng.sync()
        raw = eng.region("STAMPS", 32 * 256 * 8 * 2, dtype=torch.int64).cpu().numpy().astype(np.int64)
        phases, tot = persistent_report(raw.reshape(32, 256, 8, 2))
        for p in phases:
            print(json.dumps(p), flush=True)
        print(json.dumps({"persistent_kernel_us": tot}), flush=True)
        eng.close()
        return
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    data = torch.randint(0, 256, (4096, 3, 32, 32), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (4096,), device=dev)
    model = NetResDeep().to(dev)
    eng = NetResDeepEngine(model, data, labels, EngineConfig(batch_max=32, dtype=dtype))
    eng.set_indices(np.arange(4096, dtype=np.int32))
    eng.set_cursor(0)
    eng.run(32, 50)   # warm up, then one more step whose stamps we keep
    eng.sync()
    eng.run(32, 1)
    eng.sync()
    raw = eng.region("STAMPS", 32 * 256 * 8 * 2, dtype=torch.int64).cpu().numpy().astype(np.int64)
    st = raw.reshape(32, 256, 8, 2)
    res = {"dtype": dtype, "kernels": []}
    prev_end = None
    for k, name in enumerate(SLOTS):
        s = st[k]
        valid = s[:, 0, 1] != 0
        if not valid.any():
            continue
        s = s[valid]
        rt0 = s[:, 0, 1]
        rt5 = s[:, 5, 1]
        ok5 = rt5 != 0
        entry = {"kernel": name, "wgs": int(valid.sum()),
                 "skew_us": round((rt0.max() - rt0.min()) / 100.0, 2)}
        if ok5.any():
            entry["span_us"] = round((rt5[ok5].max() - rt0.min()) / 100.0, 2)
            entry["wg_med_us"] = round(float(np.median(rt5[ok5] - rt0[ok5])) / 100.0, 2)
            if prev_end is not None:
                entry["gap_us"] = round((rt0.min() - prev_end) / 100.0, 2)
            prev_end = rt5[ok5].max()
        phases = {}
        for a, b in ((0, 1), (1, 2), (2, 3), (3, 4), (4, 5)):
            m = (s[:, a, 0] != 0) & (s[:, b, 0] != 0)
            if m.any():
                phases[f"p{a}{b}_cyc"] = int(np.median(s[m, b, 0] - s[m, a, 0]))
        entry.update(phases)
        res["kernels"].append(entry)
        print(json.dumps(entry), flush=True)
    res["microbench_us_per_kernel"] = microbench(native.load_micro())
    print(json.dumps({"microbench_us_per_kernel": res["microbench_us_per_kernel"]}), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
