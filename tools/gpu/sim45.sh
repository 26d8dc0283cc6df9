# Multi-GPU projection from per-rank measurements on one GPU (tools/sim_ranks.py),
# configs 4 (standard) and 5 (paper, halo rows).  Usage (GPU box): TAG=r03b bash tools/gpu/sim45.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03}
: > gpurun_out/${T}_sim_ranks.jsonl
for c in 4 5; do
  timeout -k 10 300 python tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 3 >> gpurun_out/${T}_sim_ranks.jsonl 2> gpurun_out/${T}_sim_$c.err || { echo "sim $c failed"; tail gpurun_out/${T}_sim_$c.err; exit 1; }
done
cat gpurun_out/${T}_sim_ranks.jsonl
