"""Summarise rocprofv3 PMC databases (``--pmc ... -d DIR``) for the GEMM kernels of bench/gemm_shortk.py.

    python bench/pmc_summary.py --fetch gpurun_out/pmc_fetch/*.db --write gpurun_out/pmc_write/*.db \
        [--sq gpurun_out/pmc_sq/*.db] [--kernel k_gemm_stream] [--per-shape 24]

The dispatches of the chosen kernel are taken in order and grouped `--per-shape` at a time (gemm_shortk.py runs
1 + 3 + 20 calls per shape, in its SHAPES order; for k_gemm_stream only the shapes its launch rule takes: K <= 512,
M >= 16384, N % 128 == 0 or N == 64); per group the median duration and the mean counter values, with
FETCH_SIZE doubled (on gfx950 it reports half the bytes of wide coalesced streaming reads: MI355X guide) and the
achieved HBM bandwidth (FETCH + WRITE bytes over the kernel time).  One JSON line per shape.
"""
import argparse
import json
import os
import sqlite3
import statistics
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def dispatches(db: str, kernel: str) -> list:
    """[(dispatch_id, duration_ns, {counter: value})] of `kernel`, in dispatch order."""
    c = sqlite3.connect(db)
    rows = c.execute("select dispatch_id, kernel_name, counter_name, value, start, end from counters_collection "
                     "order by dispatch_id").fetchall()
    out, cur = [], {}
    for did, name, cname, val, start, end in rows:
        if kernel not in name:
            continue
        if did not in cur:
            cur[did] = (end - start, {})
            out.append(did)
        cur[did][1][cname] = cur[did][1].get(cname, 0.0) + float(val)
    return [(d, cur[d][0], cur[d][1]) for d in out]


def main() -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--fetch", required=True)
    ap.add_argument("--write", required=True)
    ap.add_argument("--sq", default=None)
    ap.add_argument("--kernel", default="k_gemm_stream")
    ap.add_argument("--per-shape", type=int, default=24)
    a = ap.parse_args()
    from gemm_shortk import SHAPES
    f, w = dispatches(a.fetch, a.kernel), dispatches(a.write, a.kernel)
    sq = dispatches(a.sq, a.kernel) if a.sq else None
    n = a.per_shape
    shapes = [s for s in SHAPES if a.kernel != "k_gemm_stream" or
              (s[2] <= 512 and s[0] >= 16384 and (s[1] % 128 == 0 or s[1] == 64))]
    for i, (M, N, K) in enumerate(shapes):
        gf, gw = f[i * n:(i + 1) * n], w[i * n:(i + 1) * n]
        if len(gf) < n or len(gw) < n:
            break
        dur_us = statistics.median([d[1] for d in gw + gf]) / 1e3  # (counter runs: durations include profiling)
        fetch_b = 2 * 1024 * statistics.mean(d[2].get("FETCH_SIZE", 0.0) for d in gf)
        write_b = 1024 * statistics.mean(d[2].get("WRITE_SIZE", 0.0) for d in gw)
        ideal = 2 * (M * K + M * N)
        rec = {"kernel": a.kernel, "shape": f"{M}x{N}x{K}", "us_median": round(dur_us, 1),
               "fetch_MB": round(fetch_b / 1e6, 1), "write_MB": round(write_b / 1e6, 1),
               "ideal_MB": round(ideal / 1e6, 1), "hbm_TBps": round((fetch_b + write_b) / dur_us / 1e6, 2)}
        if sq:
            g = sq[i * n:(i + 1) * n]
            for k in sorted(g[0][2]):
                rec[k] = round(statistics.mean(d[2][k] for d in g), 1)
        print(json.dumps(rec))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
