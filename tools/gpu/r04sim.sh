# Round-4: multi-GPU projections (tools/sim_ranks.py, placement-aware model) on the committed tree.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04sim}
: > gpurun_out/${T}.jsonl
for c in 5 4; do
  timeout -k 10 200 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 10 >> gpurun_out/${T}.jsonl 2> gpurun_out/${T}.err || { echo "sim failed"; tail gpurun_out/${T}.err; exit 1; }
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}.jsonl"):
    d = json.loads(l)
    print(d["config"], d["chunks"], d["world"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["last_chunk_place_ms"], d["frame_ms_153GBs"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
