# A/B of the paper-mode launch order: RT_PAPER_ORDER=0 (row order, no timing), 1 (timing only), 2 (costliest first).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-ab_order}
: > gpurun_out/${T}.jsonl
for rep in 1 2; do
for o in 0 2 3; do
  RT_PAPER_ORDER=$o timeout -k 10 200 python3 tools/sim_ranks.py --config 5 --worlds 1,8 --reps 10 | sed "s/^{/{\"order\": $o, /" >> gpurun_out/${T}.jsonl || exit 1
done
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}.jsonl"):
    d = json.loads(l)
    print(d["order"], d["world"], d["max_rank_wall_ms"], d["max_rank_kernel_ms"], d["min_rank_wall_ms"], d["frame_ms_153GBs"])
PY
