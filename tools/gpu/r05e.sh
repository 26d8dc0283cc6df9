# Distributed-frame tests + config-5 multi-GPU projection (cost-balanced partition).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05e}
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -k "dist or paper" > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error" gpurun_out/${T}_tests.log | head -20; tail -20 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
: > gpurun_out/${T}_sim_ranks.jsonl
for c in ${SIMCFGS:-5}; do
  timeout -k 10 400 python tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 3 >> gpurun_out/${T}_sim_ranks.jsonl 2> gpurun_out/${T}_sim_$c.err || { echo "sim $c failed"; tail gpurun_out/${T}_sim_$c.err; exit 1; }
done
python3 -c "
import json
for l in open('gpurun_out/${T}_sim_ranks.jsonl'):
    d=json.loads(l); print(d['config'], d['world'], 'max', d['max_rank_wall_ms'], 'min', d['min_rank_wall_ms'], 'r0', d['rank0_wall_ms'], 'ker', d['max_rank_kernel_ms'], 'proj', d['projected_speedup_64GBs'], d['projected_speedup_153GBs'])
"
