# Bench line per BASELINE config (2-5): value, frame ms, kernel ms, jitter ms, roofline fractions.
set -o pipefail
export TMPDIR=/tmp
for c in ${CFGS:-2 3 4 5 6}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-20} --warmup 2 > gpurun_out/bench_c$c.log 2>&1 || { echo "config $c failed"; tail gpurun_out/bench_c$c.log; exit 1; }
  tail -1 gpurun_out/bench_c$c.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print($c, d['config']['workload'], d['config']['mode'], 'value', d['value'], d['unit'], 'frame_ms', d['ms_per_step'], 'kernel_ms', r['kernel_ms'], 'rng_ms', d['wall_clock_ms']['rng'], 'frac', r['frac'], 'executed_frac', r['executed_frac'], 'rays', d['config']['rays_per_frame'], 'traced', d['config']['rays_traced_per_frame'])"
done
