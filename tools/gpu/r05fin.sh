# Round-5 evidence, part 2 (after tools/gpu/round.sh): multi-GPU projections of configs 4 and 5
# (tools/sim_ranks.py), rocprofv3 kernel stats of configs 5 and 6, the PMC passes of configs 4
# and 5 (tools/gpu/pmc_detail.sh), and the wave BVH's perf table.
# Usage (GPU box): TAG=r05g bash tools/gpu/r05fin.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05g}
: > gpurun_out/${T}_sim_ranks.jsonl
for c in 5 4; do
  timeout -k 10 200 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 10 >> gpurun_out/${T}_sim_ranks.jsonl 2> gpurun_out/${T}_sim.err || { echo "sim failed"; tail gpurun_out/${T}_sim.err; exit 1; }
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_sim_ranks.jsonl"):
    d = json.loads(l)
    print(d["config"], d["world"], d["max_rank_wall_ms"], d["max_rank_kernel_ms"], d["frame_ms_153GBs"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
for c in 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof$c -o run --output-format csv -- python3 tools/one_frame.py --config $c --frames 20 > gpurun_out/${T}_prof$c.log 2>&1 || { echo "prof $c failed"; tail gpurun_out/${T}_prof$c.log; exit 1; }
  find gpurun_out/${T}_prof$c -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats_cfg$c.csv
  head -4 gpurun_out/${T}_kernel_stats_cfg$c.csv | cut -c1-160
done
for c in 4 5; do
  timeout -k 10 400 bash tools/gpu/pmc_detail.sh $c > gpurun_out/${T}_pmc_detail_cfg$c.txt 2>&1 || { echo "pmc $c failed"; tail gpurun_out/${T}_pmc_detail_cfg$c.txt; exit 1; }
done
timeout -k 10 300 python tools/bvh_perf.py > gpurun_out/${T}_bvh_perf.txt 2>&1 || { echo "bvh perf failed"; tail gpurun_out/${T}_bvh_perf.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/${T}_bvh_perf.txt
echo done
