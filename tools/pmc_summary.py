#!/usr/bin/env python3
"""Summarize tools/gpu/pmc_frame.sh output: per-dispatch means of every
counter for the uncounted trace kernel(s) and per-wave rates."""
import collections
import csv
import glob
import json
import os
import sys


def main(src):
    per = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            per[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    out = {}
    for name, cs in per.items():
        if "rocclr" in name or "at::native" in name:
            continue
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        w = m.get("SQ_WAVES", 0.0)
        if w:
            for c in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_SMEM", "SQ_INSTS_VMEM_RD", "SQ_INSTS_VMEM_WR",
                      "SQ_INSTS_LDS", "SQ_INSTS_BRANCH", "SQ_WAVE_CYCLES"):
                if c in m:
                    m[c + "_per_wave"] = m[c] / w
        if "FETCH_SIZE" in m:
            m["fetch_bytes_x2"] = 2.0 * m["FETCH_SIZE"] * 1024
        if "WRITE_SIZE" in m:
            m["write_bytes"] = m["WRITE_SIZE"] * 1024
        # the name up to its argument list ("(anonymous namespace)" is part of
        # the qualified name, not the argument list)
        base = name.replace("(anonymous namespace)", "{anon}")
        short = base.split("(")[0].replace("{anon}", "(anonymous namespace)")[-70:]
        out[short] = {k: round(v, 3) for k, v in m.items()}
    json.dump(out, open(os.path.join(src, "summary.json"), "w"), indent=1, sort_keys=True)
    print(json.dumps(out, indent=1, sort_keys=True))


if __name__ == "__main__":
    main(sys.argv[1])
