#!/usr/bin/env python3
"""Per-rank kernel spans from a rocprofv3 kernel trace of tools/sim_ranks.py
(product path, one world): for every rt_test_dist_sim_rank call (the kernels
between two host calls are separated by idle gaps > --gap us), the span from
its first kernel start to its last kernel end, the summed kernel time, and
the per-kernel split.  Usage: python tools/rank_trace.py <kernel_trace.csv>"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    gap = float(sys.argv[2]) if len(sys.argv) > 2 else 150.0
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    calls, cur, last_end = [], [], None
    for r in rows:
        s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if last_end is not None and (s - last_end) / 1e3 > gap and cur:
            calls.append(cur)
            cur = []
        cur.append((r["Kernel_Name"], s, e))
        last_end = max(last_end or e, e)
    if cur:
        calls.append(cur)
    for i, c in enumerate(calls):
        span = (max(e for _, _, e in c) - min(s for _, s, _ in c)) / 1e3
        busy = sum(e - s for _, s, e in c) / 1e3
        per = defaultdict(float)
        for n, s, e in c:
            key = n.split("(")[0].split("::")[-1].split("<")[0]
            per[key] += (e - s) / 1e3
        top = ", ".join(f"{k} {v:.0f}" for k, v in sorted(per.items(), key=lambda kv: -kv[1])[:4])
        print(f"call {i:3d}: {len(c):3d} kernels, span {span:8.1f} us, busy {busy:8.1f} us | {top}")


if __name__ == "__main__":
    main()
