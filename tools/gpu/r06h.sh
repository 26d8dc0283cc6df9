# Full GPU suite on the in-tree build; the CLI timing and its traces; A/B lib/librtamd_head.so vs the in-tree lib.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06h_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06h_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06h_gpu_tests.log
TAG=r06h bash tools/gpu/cli_prof.sh || exit 1
for c in ${CFGS:-4 5 3 6}; do
for i in 1 2; do
for v in head cur; do
  case $v in
    cur) L=$PWD/raytracing-project_amd/lib/librtamd.so ;;
    head) L=$PWD/raytracing-project_amd/lib/librtamd_head.so ;;
  esac
  RTAMD_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-100} --warmup 3 > gpurun_out/ab_${c}_${v}_$i.json 2> gpurun_out/ab_${c}_${v}_$i.err || { echo "bench $c $v failed"; tail gpurun_out/ab_${c}_${v}_$i.err; exit 1; }
  tail -1 gpurun_out/ab_${c}_${v}_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c $v', 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'])"
done; done; done
