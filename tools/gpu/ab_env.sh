# A/B of environment settings on one library: bench frames of configs ${CFGS:-5} for each
# "VAR=value" setting given (the first run with none), alternating, twice.
# Usage (GPU box): CFGS="5" bash tools/gpu/ab_env.sh "RT_X=1" "RT_X=2" ...
set -o pipefail
export TMPDIR=/tmp
for c in ${CFGS:-5}; do
for i in 1 2; do
for v in none "$@"; do
  if [ "$v" = none ]; then E=""; else E="$v"; fi
  env $E timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-60} --warmup 3 > gpurun_out/abe_${c}_$i.json 2> gpurun_out/abe_${c}_$i.err || { echo "bench $c $v failed"; tail gpurun_out/abe_${c}_$i.err; exit 1; }
  tail -1 gpurun_out/abe_${c}_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c [$v]', 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'])"
done; done; done
