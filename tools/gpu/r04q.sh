# Round-4: chunk-count A/B of the product rank path (shared streams, paper codes) at worlds 2/4/8.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04q}
: > gpurun_out/${T}_chunks.jsonl
for n in 1 2 4; do
  for c in 5 4; do
    RT_DIST_CHUNKS=$n RT_DIST_CHUNKS_PAPER=$n timeout -k 10 200 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 10 >> gpurun_out/${T}_chunks.jsonl 2> gpurun_out/${T}.err || { echo "sim failed"; tail gpurun_out/${T}.err; exit 1; }
  done
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_chunks.jsonl"):
    d = json.loads(l)
    if d["world"] > 1:
        print(d["config"], d["chunks"], d["world"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["last_chunk_place_ms"], d["frame_ms_153GBs"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
