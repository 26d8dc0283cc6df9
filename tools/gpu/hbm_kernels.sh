# HBM bytes per launch of every kernel of a config's frame (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, one counter per
# pass, over tools/one_frame.py), with the MI355X_MICROARCH.md gfx950 corrections (FETCH x2; KiB -> B), and each
# kernel's average duration from a --kernel-trace --stats run of the same command.
# Usage (GPU box): bash tools/gpu/hbm_kernels.sh CONFIG
set -o pipefail
export TMPDIR=/tmp
C=${1:-5}
OUT=gpurun_out/hbm_c$C
rm -rf $OUT; mkdir -p $OUT
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d $OUT/$ctr -o pmc -- python3 tools/one_frame.py --config $C --frames 3 > $OUT/$ctr.log 2>&1 || { echo "$ctr pass failed"; tail -5 $OUT/$ctr.log; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 tools/one_frame.py --config $C --frames 3 > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -5 $OUT/trace.log; exit 1; }
python3 - $C <<'PY'
import csv, glob, sys, collections, re
C = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(f"gpurun_out/hbm_c{C}/{ctr}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") == ctr:
                vals[r["Kernel_Name"]][ctr].append(float(r["Counter_Value"]))
dur = {}
for f in glob.glob(f"gpurun_out/hbm_c{C}/trace/**/*kernel_stats.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        dur[r["Name"]] = (float(r["AverageNs"]) / 1e6, int(r["Calls"]))
print(f"config {C}: per launch, FETCH_SIZE x2 and WRITE_SIZE in bytes (KiB x 1024), duration = rocprofv3 average")
for k, v in vals.items():
    if "FETCH_SIZE" not in v or "WRITE_SIZE" not in v:
        continue
    fetch = 2.0 * 1024.0 * max(v["FETCH_SIZE"]); write = 1024.0 * max(v["WRITE_SIZE"])
    m = re.search(r"k_\w+(<[^>]*>)?", k); name = m.group(0) if m else k[:60]
    d = dur.get(k, (None, 0))
    bw = f"{(fetch + write) / (d[0] * 1e-3) / 1e12:.2f} TB/s" if d[0] else "-"
    print(f"  {name:55s} fetch {fetch / 1e9:8.3f} GB  write {write / 1e9:8.3f} GB  time {d[0] if d[0] else 0:8.3f} ms  {bw}")
PY
