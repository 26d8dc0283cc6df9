# Round-4: chunks-per-rank A/B through the product's rank path (configs 4, 5).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04d}
: > gpurun_out/${T}_chunks.jsonl
for n in 1 2 3 4; do
  RT_DIST_CHUNKS=$n RT_DIST_CHUNKS_PAPER=$n timeout -k 10 200 python3 tools/sim_ranks.py --config 5 --worlds 1,8 --reps 5 >> gpurun_out/${T}_chunks.jsonl 2> gpurun_out/${T}.err || { echo "sim5 failed"; tail gpurun_out/${T}.err; exit 1; }
  RT_DIST_CHUNKS=$n RT_DIST_CHUNKS_PAPER=$n timeout -k 10 200 python3 tools/sim_ranks.py --config 4 --worlds 1,8 --reps 5 >> gpurun_out/${T}_chunks.jsonl 2> gpurun_out/${T}.err || { echo "sim4 failed"; tail gpurun_out/${T}.err; exit 1; }
done
python3 - <<'PY'
import json
for l in open("gpurun_out/r04d_chunks.jsonl"):
    d = json.loads(l)
    if d["world"] == 8:
        print(d["config"], d["chunks"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["max_rank_kernel_ms"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
