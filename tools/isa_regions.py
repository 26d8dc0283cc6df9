#!/usr/bin/env python3
"""Per-source-region instruction histogram of one kernel's ISA (host-side,
no GPU).

Compiles rt_kernels_f64.hip to assembly with line tables (-gline-tables-only,
the product's flags otherwise), takes the body of the kernel whose mangled
name contains KERNEL, attributes every instruction to the innermost source
line its `.loc` names (inlined code keeps its own line), and sums instruction
classes per enclosing device function of that line:

  fp64     v_{add,mul,fma,div_*,rcp,sqrt,min,max,ldexp,frexp,...}_f64 / v_*_f64
  f32      v_*_f32 and packed v_pk_*_f32 (the cull tests)
  mov      v_mov_*, v_accvgpr_*
  cndmask  v_cndmask_*
  cmp      v_cmp_*, v_cmpx_*
  lane     v_readlane, v_readfirstlane, v_writelane, DPP / permute ops
  int      other VALU (integer, bit ops, conversions)
  salu     scalar ALU (s_*, without waitcnt / nop / branches)
  branch   s_cbranch_* / s_branch
  mem      global / buffer / scratch / flat / ds (LDS) / s_load

Static counts (each instruction once, whatever its trip count); the
dynamic VALU per wave comes from the PMC passes (tools/gpu/pmc_detail.sh).
Usage: tools/isa_regions.py [KERNEL] [--asm FILE] [--top N] [extra hipcc flags via ISA_FLAGS]
"""
import argparse
import collections
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "raytracing-project_amd")

CLASSES = ["fp64", "f32", "mov", "cndmask", "cmp", "lane", "int", "salu", "branch", "mem"]


def classify(op):
    if op.startswith(("global_", "buffer_", "scratch_", "flat_", "ds_", "s_load", "s_buffer_load", "s_store")):
        return "mem"
    if op.startswith("s_"):
        if op.startswith(("s_cbranch", "s_branch")):
            return "branch"
        if op.startswith(("s_waitcnt", "s_nop", "s_endpgm", "s_setprio", "s_barrier", "s_sleep")):
            return None
        return "salu"
    if not op.startswith("v_"):
        return None
    if op.startswith(("v_readlane", "v_readfirstlane", "v_writelane", "v_permlane", "v_bpermute", "v_swizzle")) or \
            "_dpp" in op:
        return "lane"
    if op.startswith(("v_mov", "v_accvgpr")):
        return "mov"
    if op.startswith("v_cndmask"):
        return "cndmask"
    if op.startswith(("v_cmp", "v_cmpx")):
        return "cmp"
    if op.endswith("_f64") or "_f64_" in op or op.startswith(("v_div_fmas_f64", "v_div_scale_f64", "v_div_fixup_f64")):
        return "fp64"
    if "_f32" in op or op.startswith("v_pk_"):
        return "f32"
    return "int"


FUNC_RE = re.compile(r"^\s*(?:template\s*<.*>\s*)?(?:__device__|__global__|__host__ __device__)[^;{]*?\b([A-Za-z_][A-Za-z0-9_]*)\s*\(")


def func_starts(path):
    """(line, name) of every device function definition in a source file."""
    out = []
    try:
        with open(path) as f:
            lines = f.readlines()
    except OSError:
        return out
    for i, l in enumerate(lines, 1):
        m = FUNC_RE.match(l)
        if m and not l.rstrip().endswith(";"):
            out.append((i, m.group(1)))
    return out


def region(starts, line):
    name = "?"
    for ln, nm in starts:
        if ln <= line:
            name = nm
        else:
            break
    return name


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("kernel", nargs="?", default="k_std_leanILb0ELi1E")
    ap.add_argument("--asm", default=None, help="existing assembly (skip the compile)")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--lines", action="store_true", help="also list the top source lines")
    a = ap.parse_args()
    asm = a.asm or "/tmp/isa_regions.s"
    if not a.asm:
        cmd = ["/opt/rocm/bin/hipcc", "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950", "-ffp-contract=off",
               "-fno-fast-math", "-munsafe-fp-atomics", "-mllvm", "--amdgpu-set-wave-priority", "-mllvm",
               "--structurizecfg-skip-uniform-regions", "-gline-tables-only", "-I../include", "-Icsrc/host",
               "-Icsrc/device", "--cuda-device-only", "-S", "csrc/device/rt_kernels_f64.hip", "-o", asm]
        cmd += os.environ.get("ISA_FLAGS", "").split()
        subprocess.run(cmd, cwd=PKG, check=True, stderr=subprocess.DEVNULL)
    files = {}
    per_line = collections.defaultdict(collections.Counter)
    inside = False
    cur = (None, 0)
    pat = re.compile(r"^_Z\S*" + re.escape(a.kernel) + r"\S*:")
    with open(asm) as f:
        for raw in f:
            if raw.startswith("\t.file"):
                m = re.match(r'\t\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', raw)
                if m:
                    d, n = m.group(2), m.group(3)
                    path = os.path.join(d, n) if n else d
                    files[int(m.group(1))] = path if os.path.isabs(path) else os.path.join(PKG, path)
                continue
            if not inside:
                if pat.match(raw):
                    inside = True
                continue
            if raw.startswith("\t.end_amdhsa_kernel") or raw.startswith(".Lfunc_end"):
                break
            if raw.startswith("\t.loc"):
                p = raw.split()
                cur = (int(p[1]), int(p[2]))
                continue
            if not raw.startswith("\t") or raw.startswith("\t."):
                continue
            op = raw.split()[0]
            c = classify(op)
            if c:
                per_line[cur][c] += 1
    if not per_line:
        print(f"kernel {a.kernel} not found in {asm}", file=sys.stderr)
        return 1
    starts_cache = {}
    per_region = collections.defaultdict(collections.Counter)
    for (fid, ln), cnt in per_line.items():
        path = files.get(fid, "?")
        if path not in starts_cache:
            starts_cache[path] = func_starts(path)
        key = f"{os.path.basename(path)}:{region(starts_cache[path], ln)}"
        per_region[key].update(cnt)
    total = collections.Counter()
    for c in per_region.values():
        total.update(c)
    hdr = f"{'region':44s} " + " ".join(f"{c:>7s}" for c in CLASSES) + "   valu"
    print(f"# {a.kernel}: static instructions per source region (innermost inlined function)")
    print(hdr)
    def valu(c):
        return sum(c[k] for k in ("fp64", "f32", "mov", "cndmask", "cmp", "lane", "int"))
    rows = sorted(per_region.items(), key=lambda kv: -valu(kv[1]))
    for k, c in rows[:a.top]:
        print(f"{k[:44]:44s} " + " ".join(f"{c[x]:7d}" for x in CLASSES) + f" {valu(c):6d}")
    print(f"{'TOTAL':44s} " + " ".join(f"{total[x]:7d}" for x in CLASSES) + f" {valu(total):6d}")
    if a.lines:
        print("\n# top source lines by VALU")
        for (fid, ln), c in sorted(per_line.items(), key=lambda kv: -valu(kv[1]))[:a.top]:
            print(f"{os.path.basename(files.get(fid, '?'))}:{ln:5d} " + " ".join(f"{c[x]:5d}" for x in CLASSES))
    return 0


if __name__ == "__main__":
    sys.exit(main())
