"""Same-operand GEMM workload for PMC comparisons: our bf16 GEMM (ops.gemm, default dispatch) and the library
(torch.matmul = hipBLASLt) on identical random operands, each run `--iters` times after a warm-up, so a
``rocprofv3 --pmc ...`` run over this script collects both kernels' counters in one process.

    rocprofv3 --pmc SQ_WAVE_CYCLES ... --output-format csv -d DIR -- python bench/gemm_pmc.py --shape 4096x4096x4096
    python bench/gemm_pmc.py --summarize DIR/...counter_collection.csv

--summarize: per kernel name, the median duration and the mean of each counter over its dispatches (one JSON line
per kernel).  Without rocprofv3 the script prints the event-timed us / TFLOP/s of both.
"""
import argparse
import csv
import json
import os
import statistics
import sys
from collections import defaultdict

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def summarize(paths):
    per = defaultdict(lambda: defaultdict(dict))  # kernel -> dispatch -> {counter: value, "_ns": dur}
    for p in paths:
        with open(p) as f:
            for row in csv.DictReader(f):
                k = row.get("Kernel_Name", "?")
                d = row.get("Dispatch_Id") or row.get("Correlation_Id")
                name = row.get("Counter_Name")
                val = float(row.get("Counter_Value", 0.0))
                rec = per[k][d]
                rec[name] = rec.get(name, 0.0) + val
                if "Start_Timestamp" in row and "End_Timestamp" in row:
                    rec["_ns"] = float(row["End_Timestamp"]) - float(row["Start_Timestamp"])
    for k, ds in per.items():
        recs = list(ds.values())
        names = sorted({n for r in recs for n in r if n != "_ns"})
        out = {"kernel": k[:90], "dispatches": len(recs)}
        durs = [r["_ns"] for r in recs if "_ns" in r]
        if durs:
            out["us_median"] = round(statistics.median(durs) / 1e3, 2)
        for n in names:
            out[n] = round(statistics.mean(r.get(n, 0.0) for r in recs), 1)
        print(json.dumps(out), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", default="4096x4096x4096")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--which", default="both", choices=["both", "ours", "lib"])
    ap.add_argument("--conv", default=None, help="NxHxCxCO: a 3x3 / pad-1 implicit convolution instead")
    ap.add_argument("--summarize", nargs="*", default=None)
    ap.add_argument("--zeros", action="store_true", help="zero-filled operands (DVFS comparison only)")
    a = ap.parse_args()
    if a.summarize is not None:
        summarize(a.summarize)
        return
    import torch
    from distributeddataparallel_cifar10_amd import ops
    dev = torch.device("cuda", 0)
    bf = torch.bfloat16
    torch.manual_seed(0)
    if a.conv:
        from distributeddataparallel_cifar10_amd.ops import functional as F
        n, h, c, co = (int(v) for v in a.conv.split("x"))
        x = torch.randn(n, h, h, c, device=dev).to(bf)
        wt = torch.randn(co, c, 3, 3, device=dev) * 0.05
        geo = F._geom(x, wt, 1, 1)
        wm = F._weight_matrix(wt, geo.K)
        M, N, K = n * geo.Ho * geo.Wo, co, geo.K
        ours = lambda: ops.gemm(x, wm, conv=1, geom=geo, mnk=(M, N, K), out_dtype=bf)  # noqa: E731
        xn = x.permute(0, 3, 1, 2)
        wn = wt.to(bf).contiguous(memory_format=torch.channels_last)
        lib = lambda: torch.nn.functional.conv2d(xn, wn, stride=1, padding=1)  # noqa: E731
    else:
        M, N, K = (int(v) for v in a.shape.split("x"))
        x = torch.randn(M, K, device=dev).to(bf)
        w = torch.randn(N, K, device=dev).to(bf)
        if a.zeros:
            x.zero_()
            w.zero_()
        ours = lambda: ops.gemm(x, w, out_dtype=bf)  # noqa: E731
        lib = lambda: torch.matmul(x, w.t())  # noqa: E731
        y = ours().float()
        ref = x.float() @ w.float().t()
        print(json.dumps({"rel_err": ((y - ref).norm() / ref.norm().clamp_min(1e-30)).item()}), flush=True)
        del y, ref
    fns = {"ours": ours, "lib": lib}
    for name in (["ours", "lib"] if a.which == "both" else [a.which]):
        fn = fns[name]
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(a.iters):
            fn()
        e1.record()
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) * 1e3 / a.iters
        print(json.dumps({"which": name, "shape": f"{M}x{N}x{K}", "us": round(us, 1),
                          "tflops": round(2 * M * N * K / us / 1e6, 1)}), flush=True)


if __name__ == "__main__":
    main()
