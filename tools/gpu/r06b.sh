# Config 2 / 3: the wave-level culling threshold (RT_WV_MIN) A/B, interleaved, twice; parity subset under RT_WV_MIN=1 first.
set -o pipefail
export TMPDIR=/tmp
RT_WV_MIN=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06b_par_wv1.log 2>&1 || { echo "parity (RT_WV_MIN=1) failed"; tail -30 gpurun_out/r06b_par_wv1.log; exit 1; }
tail -1 gpurun_out/r06b_par_wv1.log
for i in 1 2; do
for c in 2 3; do
for w in 4 3 2 1; do
  RT_WV_MIN=$w timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps 100 --warmup 3 > gpurun_out/r06b_${c}_$w.json 2> gpurun_out/r06b_${c}_$w.err || { echo "bench $c $w failed"; tail gpurun_out/r06b_${c}_$w.err; exit 1; }
  tail -1 gpurun_out/r06b_${c}_$w.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c wvmin $w', d['roofline']['kernel'], 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])"
done; done; done
