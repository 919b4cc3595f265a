"""Where does the sliced persistent step spend its time?  (diagnostic; needs the stamps build, -DDCA_STAMPS)

Runs the image-sliced engine (csrc/netresdeep_pks.hip) built with in-kernel s_memtime / s_memrealtime stamps
(thread 0 of every workgroup, DCA_STAMP slots) and prints per-phase medians over the workgroups, plus the
exchange statistics of the detailed forward / backward blocks (DCA_DETAIL_FWD / DCA_DETAIL_BWD, default 5):
publication spread, last publication -> done, publication -> done.

    python bench/stamps_pks.py [bf16|fp32]
"""
from __future__ import annotations

import json
import os
import sys

os.environ.setdefault("DCA_ENGINE_VARIANT", "stamps")
import numpy as np  # noqa: E402
import torch  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from model.resnet import NetResDeep  # noqa: E402
from distributeddataparallel_cifar10_amd.runtime.engine import EngineConfig, NetResDeepEngine  # noqa: E402


def stamp(st, slot, k):
    """realtime (10 ns ticks) and memtime (cycles) of stamp (slot, k) per valid workgroup."""
    return st[slot, :, k, 1].astype(np.int64), st[slot, :, k, 0].astype(np.int64)


def main():
    dtype = sys.argv[1] if len(sys.argv) > 1 else "bf16"
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    data = torch.randint(0, 256, (4096, 3, 32, 32), dtype=torch.uint8, device=dev)
    labels = torch.randint(0, 10, (4096,), device=dev)
    eng = NetResDeepEngine(NetResDeep().to(dev), data, labels, EngineConfig(batch_max=32, dtype=dtype))
    assert eng.kind_name == "sliced", eng.kind_name
    eng.set_indices(np.arange(4096, dtype=np.int32))
    eng.set_cursor(0)
    eng.run(32, 60)
    eng.sync()
    eng.run(32, 1, False)  # one eager step: its stamps are kept
    eng.sync()
    raw = eng.region("STAMPS", 32 * 256 * 8 * 2, dtype=torch.int64).cpu().numpy().astype(np.int64)
    st = raw.reshape(32, 256, 8, 2)
    G = 128
    st = st[:, :G]
    seq = [("start", (0, 0)), ("stem.staged", (0, 2)), ("stem.mfma", (0, 3)), ("stem.end", (0, 1))]
    seq += [(f"fwd{i}", (1 + i // 8, i % 8)) for i in range(10)]
    seq += [("head.fc1part", (3, 1)), ("head.xchg", (3, 2)), ("head.ce", (3, 3)), ("head.end", (3, 0))]
    seq += [(f"bwd{9 - k}", (4 + k // 8, k % 8)) for k in range(10)]
    seq += [("end.wgrad0", (5, 2)), ("end.stem_staged", (5, 3)), ("end.stem_wgrad", (5, 4)), ("end", (5, 7))]
    prev = None
    total = 0.0
    for name, (sl, k) in seq:
        rt, _ = stamp(st, sl, k)
        if prev is not None:
            d = np.median(rt - prev) / 100.0
            total += d
            print(json.dumps({"phase": name, "us": round(float(d), 2)}), flush=True)
        prev = rt
    rt0, _ = stamp(st, 0, 0)
    rte, _ = stamp(st, 5, 7)
    print(json.dumps({"kernel_us_median_wg": round(float(np.median(rte - rt0)) / 100.0, 2),
                      "start_skew_us": round(float(rt0.max() - rt0.min()) / 100.0, 2),
                      "span_us": round(float(rte.max() - rt0.min()) / 100.0, 2), "dtype": dtype}), flush=True)
    # detailed blocks: forward slot 6 (0 conv, 1 published, 2 exchange done, 3 barrier), previous = fwd block end
    for label, slot, prev_stamp, npts, pub, done in (("fwd", 6, (1, 4), 4, 1, 2), ("bwd", 7, (4, 3), 7, 1, 4)):
        p0, _ = stamp(st, *prev_stamp)
        pts = [stamp(st, slot, j)[0] for j in range(npts)]
        seg = [np.median(pts[0] - p0)] + [np.median(pts[j] - pts[j - 1]) for j in range(1, npts)]
        print(json.dumps({"detail": label + "5", "us": [round(float(x) / 100.0, 2) for x in seg]}), flush=True)
        P, D = pts[pub], pts[done]
        print(json.dumps({"xchg": label + "5", "pub_spread_us": round(float(P.max() - P.min()) / 100.0, 2),
                          "last_pub_to_done_med_us": round(float(np.median(D) - P.max()) / 100.0, 2),
                          "last_pub_to_first_done_us": round(float(D.min() - P.max()) / 100.0, 2),
                          "done_spread_us": round(float(D.max() - D.min()) / 100.0, 2),
                          "pub_to_done_med_us": round(float(np.median(D - P)) / 100.0, 2)}), flush=True)
    # reduction kernel (slot 8, workgroup = gradient segment): 0 start, 1 segment summed, 2 exchanged, 3 end;
    # fc workers of the step kernel (slot 9, fc1 block 0..63, 64 = fc tail): 0 start, 1 head seen + computed, ...
    red = raw.reshape(32, 256, 8, 2)[8]
    step_end = rte.max()
    # seg_layout(128) with the fc segments on the fc workers: 72 trunk chunks, 9 conv1 chunks, the BN tail
    groups = {"trunk": range(0, 72), "stem": range(72, 81), "bn_tail": range(81, 82)}
    r0 = red[:82, 0, 1].astype(np.int64)
    r3 = red[:82, 3, 1].astype(np.int64)
    if (r0 != 0).all():
        print(json.dumps({"reduce_gap_after_step_us": round(float(r0.min() - step_end) / 100.0, 2),
                          "reduce_span_us": round(float(r3.max() - r0.min()) / 100.0, 2),
                          "reduce_start_skew_us": round(float(r0.max() - r0.min()) / 100.0, 2)}), flush=True)
        for g, idx in groups.items():
            x = red[list(idx)].astype(np.int64)
            seg = [np.median(x[:, j + 1, 1] - x[:, j, 1]) / 100.0 for j in range(3)]
            print(json.dumps({"reduce": g, "sum_us": round(float(seg[0]), 2), "exchange_us": round(float(seg[1]), 2),
                              "sgd_us": round(float(seg[2]), 2),
                              "end_after_first_start_us": round(float(x[:, 3, 1].max() - r0.min()) / 100.0, 2)}),
                  flush=True)
    fcw = raw.reshape(32, 256, 8, 2)[9][:65].astype(np.int64)
    if (fcw[:, 3, 1] != 0).all():
        print(json.dumps({"fc_workers": 65, "compute_us": round(float(np.median(fcw[:, 1, 1] - fcw[:, 0, 1])) / 100.0, 2),
                          "last_end_before_step_end_us": round(float(step_end - fcw[:, 3, 1].max()) / 100.0, 2)}),
              flush=True)
    eng.close()


if __name__ == "__main__":
    main()
