# Round-4: distributed-frame GPU tests + chunk A/B on the rotated, root-weighted partition.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04e}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_jitter_rows.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_chunks.jsonl
for n in 2 3 4; do
  for c in 5 4; do
    RT_DIST_CHUNKS=$n RT_DIST_CHUNKS_PAPER=$n timeout -k 10 200 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 10 >> gpurun_out/${T}_chunks.jsonl 2> gpurun_out/${T}.err || { echo "sim failed"; tail gpurun_out/${T}.err; exit 1; }
  done
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04e_chunks.jsonl"):
    d = json.loads(l)
    if d["world"] > 1:
        print(d["config"], d["chunks"], d["world"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["max_rank_kernel_ms"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
