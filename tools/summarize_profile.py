#!/usr/bin/env python3
"""Summarize rocprofv3 CSVs of tools/profile_bench.sh into profiles/<tag>_*.

Writes profiles/<tag>_kernel_stats.csv (rocprofv3 --stats output, verbatim),
profiles/<tag>_pmc.json (counters per kernel, per dispatch) and
profiles/traffic.json (HBM bytes per launch of the trace kernel, from
FETCH_SIZE x 2 (gfx950 calibration, MI355X_MICROARCH.md §HBM) + WRITE_SIZE, KiB -> B).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def main(src, dst, tag):
    os.makedirs(dst, exist_ok=True)
    stats = glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if stats:
        shutil.copy(stats[0], os.path.join(dst, f"{tag}_kernel_stats.csv"))
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "pmc_*", "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            per[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    pmc = {}
    for name, cs in per.items():
        if "rocclr" in name or "at::native" in name:
            continue
        pmc[name] = {c: sum(v) / len(v) for c, v in cs.items()}   # mean per dispatch
    json.dump(pmc, open(os.path.join(dst, f"{tag}_pmc.json"), "w"), indent=1, sort_keys=True)
    def uncounted_trace(n):
        # the timed trace kernel: k_std_lean<C, WV> / k_std<E, D, SEC, C, WV> with C = false
        for key, pos in (("k_std_lean<", 0), ("k_std<", 3)):
            if key in n:
                args = [a.strip() for a in n.split(key, 1)[1].split(">", 1)[0].split(",")]
                return len(args) > pos and args[pos] == "false"
        return False

    cands = [n for n in pmc if uncounted_trace(n)]
    main_k = max(cands, key=lambda n: pmc[n].get("SQ_WAVES", 0.0)) if cands else None
    if main_k and "FETCH_SIZE" in pmc[main_k] and "WRITE_SIZE" in pmc[main_k]:
        f, w = pmc[main_k]["FETCH_SIZE"], pmc[main_k]["WRITE_SIZE"]
        out = {"config": 4, "kernel": main_k, "fetch_kib_raw": f, "write_kib": w,
               "hbm_bytes_per_launch": (2.0 * f + w) * 1024.0,
               "note": "FETCH_SIZE doubled per the gfx950 calibration for wide streaming reads; "
                       "this kernel's reads are mostly scalar-cache and 16-B jitter loads, so the read side is "
                       "an upper estimate"}
        json.dump(out, open(os.path.join(dst, "traffic.json"), "w"), indent=1)
        print(json.dumps(out))
    print("kernels:", list(pmc))


if __name__ == "__main__":
    main(*sys.argv[1:4])
