# Round-4: paper finish with up-front loads (no hit array): paper tests, config-5 kernel stats, sims.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04x}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py tests/test_gpu_crowd.py tests/test_gpu_fp32.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof5 -o run --output-format csv -- python3 tools/one_frame.py --config 5 --frames 20 > gpurun_out/${T}_prof5.log 2>&1 || { echo "prof failed"; tail gpurun_out/${T}_prof5.log; exit 1; }
python3 - <<PY
import csv, glob
f = glob.glob("gpurun_out/${T}_prof5/**/*kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    print(r["Name"][:60], r["Calls"], r["AverageNs"])
PY
: > gpurun_out/${T}_sim.jsonl
timeout -k 10 200 python3 tools/sim_ranks.py --config 5 --worlds 1,8 --reps 10 >> gpurun_out/${T}_sim.jsonl 2> gpurun_out/${T}_sim.err || { echo "sim failed"; tail gpurun_out/${T}_sim.err; exit 1; }
python3 - <<PY
import json
for l in open("gpurun_out/${T}_sim.jsonl"):
    d = json.loads(l)
    print(d["config"], d["chunks"], d["world"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["max_rank_kernel_ms"], d["frame_ms_153GBs"], d["projected_speedup_153GBs"])
PY
