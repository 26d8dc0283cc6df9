# Root-shed A/B of the paper partition (RT_ROOT_SHED_PAPER per mille per rank; product default 30):
# config-5 projections at 8 ranks (tools/sim_ranks.py) for each value given.
# Usage (GPU box): bash tools/gpu/shed.sh 30 45 60
set -o pipefail
export TMPDIR=/tmp
: > gpurun_out/shed.jsonl
for v in "$@"; do
  RT_ROOT_SHED_PAPER=$v timeout -k 10 200 python3 tools/sim_ranks.py --config 5 --worlds ${WORLDS:-8} --reps 10 > gpurun_out/shed_$v.jsonl 2> gpurun_out/shed_$v.err || { echo "sim $v failed"; tail gpurun_out/shed_$v.err; exit 1; }
  python3 -c "
import json,sys
for l in open('gpurun_out/shed_$v.jsonl'):
    d=json.loads(l); d['shed']=$v; print(json.dumps(d), file=open('gpurun_out/shed.jsonl','a'))
    print('shed $v world', d['world'], 'frame', d['frame_ms_153GBs'], 'x', d['projected_speedup_153GBs'], 'ranks', d['rank_wall_ms'])
"
done
