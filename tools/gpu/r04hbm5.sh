# Round-4: HBM traffic of config 5's paper kernels (rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE, separate passes).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04hbm5}
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${T}_fetch -o run -- python3 tools/one_frame.py --config 5 --frames 3 > gpurun_out/${T}_fetch.log 2>&1 || { echo "fetch pass failed"; tail gpurun_out/${T}_fetch.log; exit 1; }
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/${T}_write -o run -- python3 tools/one_frame.py --config 5 --frames 3 > gpurun_out/${T}_write.log 2>&1 || { echo "write pass failed"; tail gpurun_out/${T}_write.log; exit 1; }
python3 - <<PY
import csv, glob, collections
for tag in ("fetch", "write"):
    f = glob.glob("gpurun_out/${T}_%s/**/*counter_collection.csv" % tag, recursive=True)[0]
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for (k, c), v in sorted(acc.items()):
        print(tag, c, k, "per launch (raw):", sum(v) / len(v) if v else 0, "n=", len(v))
PY
