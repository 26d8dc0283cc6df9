# Three default bench runs' CLI lines (driver-like cli_total, cli_split, cli_setup).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05cli}
for i in 1 2 3; do
  timeout -k 10 90 python bench.py --no-cpu --no-pmc --fp32-steps 0 --steps 3 --warmup 1 > gpurun_out/${T}_cli_$i.json 2>&1 || { tail gpurun_out/${T}_cli_$i.json; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/${T}_cli_$i.json').read().strip().splitlines()[-1]); w=d['wall_clock_ms']; print(json.dumps({'cli_total': w['cli_total'], 'cli_split': w['cli_split'], 'cli_setup': w['cli_setup']}))"
done
