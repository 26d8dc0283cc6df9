set -o pipefail
export TMPDIR=/tmp
for c in 2 3 4 5; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --steps 3 --warmup 1 > gpurun_out/bench_c$c.log 2>&1 || { echo "config $c failed"; tail gpurun_out/bench_c$c.log; exit 1; }
  tail -1 gpurun_out/bench_c$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print($c, d['value'], d['ms_per_step'], d['config']['width'], d['config']['height'], d['config']['mode'], d['roofline']['kernel_ms'], d['rng_ms'], d['roofline']['frac'], d['roofline']['executed_frac'])"
done
