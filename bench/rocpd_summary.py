"""Summarise a rocprofv3 kernel-trace database (rocpd SQLite): per-kernel duration statistics and the gaps
between consecutive dispatches of the persistent training step.

    python bench/rocpd_summary.py gpurun_out/prof_pk/run_results.db > profiles/rocprof_persistent_summary.txt
"""
from __future__ import annotations

import collections
import os
import sqlite3
import statistics
import sys


def main(path: str) -> None:
    c = sqlite3.connect(path)
    rows = list(c.execute("select name, start, end, grid_x, workgroup_x, lds_size, vgpr_count, sgpr_count, "
                          "scratch_size from kernels order by start"))
    by = collections.defaultdict(list)
    meta = {}
    for n, s, e, gx, wx, lds, vg, sg, scr in rows:
        by[n].append((e - s) / 1e3)
        meta[n] = (gx, wx, lds, vg, sg, scr)
    grand = sum(sum(v) for v in by.values()) or 1.0
    print(f"{'kernel':60s} {'calls':>6s} {'total_ms':>9s} {'pct':>5s} {'median_us':>10s} {'p10_us':>8s} {'p90_us':>8s} "
          f"{'grid':>6s} {'wg':>5s} {'lds':>7s} {'vgpr':>5s} {'sgpr':>5s} {'scratch':>7s}")
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        v.sort()
        gx, wx, lds, vg, sg, scr = meta[n]
        print(f"{n[:60]:60s} {len(v):6d} {sum(v) / 1e3:9.2f} {100 * sum(v) / grand:5.1f} {v[len(v) // 2]:10.2f} {v[len(v) // 10]:8.2f} {v[9 * len(v) // 10]:8.2f} "
              f"{gx:6d} {wx:5d} {lds:7d} {vg:5d} {sg:5d} {scr:7d}")
    seq = [(n, s, e) for n, s, e, *_ in rows if "k_pks_step" in n or "k_pks_reduce" in n]
    if len(seq) > 20:
        gaps = [(b[1] - a[2]) / 1e3 for a, b in zip(seq, seq[1:])]
        steps = [i for i, r in enumerate(seq) if "k_pks_step" in r[0]]
        per = [(seq[b][1] - seq[a][1]) / 1e3 for a, b in zip(steps, steps[1:])]
        print(f"\npersistent step: period median {statistics.median(per):.2f} us over {len(per)} steps; "
              f"dispatch gap median {statistics.median(gaps):.2f} us, max {max(gaps):.2f} us")


if __name__ == "__main__":
    if len(sys.argv) != 2 or sys.argv[1].startswith("-") or not os.path.isfile(sys.argv[1]):
        sys.exit(__doc__)  # (sqlite3.connect would create an empty database at a wrong path)
    main(sys.argv[1])
