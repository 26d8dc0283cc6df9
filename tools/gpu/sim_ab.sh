# Multi-GPU projection A/B (tools/sim_ranks.py, one GPU): paper / standard chunk counts and root shed.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r06s}_sim_ab.jsonl
: > $OUT
for ch in 4 2 3 1; do
  RT_DIST_CHUNKS_PAPER=$ch timeout -k 10 300 python tools/sim_ranks.py --config 5 --worlds 1,4,8 > gpurun_out/sim_tmp.jsonl 2> gpurun_out/sim_tmp.err || { echo "sim cfg5 ch$ch failed"; tail gpurun_out/sim_tmp.err; exit 1; }
  python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), ab='chunks_paper=$ch'))) for l in open('gpurun_out/sim_tmp.jsonl') if l.startswith('{')]" >> $OUT
done
for ch in 4 3 2; do
  RT_DIST_CHUNKS=$ch timeout -k 10 300 python tools/sim_ranks.py --config 4 --worlds 1,8 > gpurun_out/sim_tmp.jsonl 2> gpurun_out/sim_tmp.err || { echo "sim cfg4 ch$ch failed"; tail gpurun_out/sim_tmp.err; exit 1; }
  python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), ab='chunks_std=$ch'))) for l in open('gpurun_out/sim_tmp.jsonl') if l.startswith('{')]" >> $OUT
done
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); print(d['ab'], 'cfg', d['config'], 'world', d['world'], 'max_wall', d['max_rank_wall_ms'], 'r0', d['rank0_wall_ms'], 'kmax', d['max_rank_kernel_ms'], 'x64', d['projected_speedup_64GBs'], 'x153', d['projected_speedup_153GBs'])"
