# Frame-path check: dist/jitter/CLI/parity GPU tests, then the config-4 bench line (frame ms, rng, kernel) for the
# in-tree library and lib/exp variants.  Usage (GPU box): bash tools/gpu/frame_ab.sh name1 ...
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_jitter_rows.py tests/test_gpu_parity.py tests/test_gpu_cli.py -x -q --timeout 120 --timeout-method thread > gpurun_out/frame_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/frame_tests.log; exit 1; }
tail -1 gpurun_out/frame_tests.log
for v in cur "$@"; do
  if [ $v = cur ]; then L=$PWD/raytracing-project_amd/lib/librtamd.so; else L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so; fi
  RTAMD_LIB=$L timeout -k 10 200 python bench.py --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-100} --warmup 3 > gpurun_out/frame_$v.json 2> gpurun_out/frame_$v.err || { echo "bench $v failed"; tail gpurun_out/frame_$v.err; exit 1; }
  tail -1 gpurun_out/frame_$v.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); w=d['wall_clock_ms']; print('$v', 'value', d['value'], 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'rng_ms', w['rng'], 'frac', d['roofline']['frac'])"
done
