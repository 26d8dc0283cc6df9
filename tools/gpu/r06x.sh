# Multi-GPU projection of config 5 with the plain paper kernel: paper chunk counts 2 (default), 1, 3 at worlds 1 and 8.
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/r06x_sim_ab.jsonl
: > $OUT
for ch in 2 1 3 2; do
  RT_DIST_CHUNKS_PAPER=$ch timeout -k 10 300 python tools/sim_ranks.py --config 5 --worlds 1,8 > gpurun_out/sim_tmp.jsonl 2> gpurun_out/sim_tmp.err || { echo "sim cfg5 ch$ch failed"; tail gpurun_out/sim_tmp.err; exit 1; }
  python3 -c "import json,sys; [print(json.dumps(dict(json.loads(l), ab='chunks_paper=$ch'))) for l in open('gpurun_out/sim_tmp.jsonl') if l.startswith('{')]" >> $OUT
done
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); print(d['ab'], 'cfg', d['config'], 'world', d['world'], 'max_wall', d['max_rank_wall_ms'], 'r0', d['rank0_wall_ms'], 'kmax', d['max_rank_kernel_ms'], 'x64', d['projected_speedup_64GBs'], 'x153', d['projected_speedup_153GBs'])"
