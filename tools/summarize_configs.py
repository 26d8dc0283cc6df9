#!/usr/bin/env python3
"""Per-config evidence table from one evidence run (tools/gpu/r06_evidence.sh):
the bench line of each config (gpurun_out/<TAG>_bench_c<C>.json), the rocprofv3
average of its trace kernel(s) (<TAG>_prof_c<C>/run_kernel_stats.csv) and the
PMC instruction mix per wave (<TAG>_pmc_c<C>.txt).
Usage: python tools/summarize_configs.py TAG > profiles/<file>.txt"""
import csv
import json
import os
import re
import sys

TAG = sys.argv[1] if len(sys.argv) > 1 else "r06f"
D = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "gpurun_out")
NAMES = {2: "config 2", 3: "config 3", 4: "config 4", 5: "config 5", 6: "recursion row"}


def bench(c):
    lines = open(os.path.join(D, f"{TAG}_bench_c{c}.json")).read().strip().splitlines()
    return json.loads(lines[-1])


def prof(c):
    out = {}
    for r in csv.DictReader(open(os.path.join(D, f"{TAG}_prof_c{c}", "run_kernel_stats.csv"))):
        out[r["Name"]] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
    return out


def pmc(c):
    blocks, cur = {}, None
    for line in open(os.path.join(D, f"{TAG}_pmc_c{c}.txt")):
        if not line.startswith(" "):
            cur = line.strip()
            blocks[cur] = {}
        else:
            m = re.match(r"\s+(\S+)\s+\S+\s+\(n=\d+\)\s+per wave (\S+)", line)
            if m and cur is not None:
                blocks[cur][m.group(1)] = float(m.group(2))
    return blocks


def short(name):
    m = re.search(r"k_\w+<[^>]*>|k_\w+", name)
    return m.group(0) if m else name


print(f"# Per-config evidence, one tree, one gpurun call (tools/gpu/r06_evidence.sh TAG={TAG}), summarized by")
print("# tools/summarize_configs.py: the 100-frame bench line (bench.py --config C), the rocprofv3 average of its")
print("# trace kernel over a 30-frame run, and the PMC instruction mix per wave (4 counter passes).  frac = SURVEY 8d")
print("# FLOP model x the reference's own primitive calls / kernel time / 78.6 TF; executed = the FLOPs the kernel ran")
print("# after culling.  FP64 ops = ADD + MUL + FMA + TRANS F64 instructions per wave.")
for c in (2, 3, 4, 5, 6):
    try:
        b, p, m = bench(c), prof(c), pmc(c)
    except OSError as e:
        print(f"\nconfig {c}: missing ({e})")
        continue
    r = b["roofline"]
    k = r["kernel"]
    kshort = short(k)
    print(f"\n{NAMES[c]}: {b['config']['workload']} [{b['config']['mode']}]")
    occ = r.get("occupancy", {})
    rp = [(n, v) for n, v in p.items() if kshort.split("<")[0] in n and "<false" in n]
    rps = ", ".join(f"{short(n)} {v[0]:.3f} ms x {v[1]}" for n, v in rp)
    print(f"  kernel {k}: bench HIP events {r['kernel_ms']:.3f} ms; rocprofv3 {rps}")
    if b["config"]["mode"] == "paper":
        fin = [(n, v) for n, v in p.items() if "k_paper_finish" in n]
        print("  (paper: bench kernel ms = primary + finish; " +
              ", ".join(f"{short(n)} {v[0]:.3f} ms x {v[1]}" for n, v in fin) + ")")
    wc = b.get("wall_clock_ms") or {}
    print(f"  jitter {wc.get('rng', 0.0):.3f} ms, frame {b['ms_per_step']:.3f} ms, {b['value']:,.0f} Mrays/s "
          f"(reference-defined {b['config']['rays_per_frame']:,} rays/frame, traced {b['config']['rays_traced_per_frame']:,})")
    print(f"  FLOP-model frac {r['frac']:.4f}, executed frac {r.get('executed_frac', 0.0):.4f}; occupancy: "
          f"{occ.get('vgprs')} VGPRs, {occ.get('scratch_bytes_per_lane')} B scratch, {occ.get('lds_bytes')} B LDS, "
          f"{occ.get('waves_per_simd')} waves/SIMD")
    for name, v in m.items():
        if ("k_std" in name or "k_paper_primary" in name) and "<false" in name and "SQ_INSTS_VALU" in v:
            f64 = sum(v.get(x, 0.0) for x in ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64",
                                               "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64"))
            print(f"  per wave ({name.strip()[:60]}...): VALU {v['SQ_INSTS_VALU']:,.0f} (FP64 ops {f64:,.0f}), "
                  f"SALU {v.get('SQ_INSTS_SALU', 0.0):,.0f}, LDS {v.get('SQ_INSTS_LDS', 0.0):,.0f}")
