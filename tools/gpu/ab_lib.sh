# A/B of library builds: lib/librtamd_head.so (the previous build, copied there by hand), the in-tree
# lib/librtamd.so ("cur") and lib/exp/librtamd_<name>.so for each name given.  Parity subset on the
# in-tree build first, then bench frames of configs ${CFGS:-4 5 6}, the variants alternating, twice.
# Usage (GPU box): CFGS="4 5" bash tools/gpu/ab_lib.sh [name ...]
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py tests/test_gpu_bvh.py tests/test_gpu_recursion.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ab_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/ab_tests.log; exit 1; }
tail -1 gpurun_out/ab_tests.log
for c in ${CFGS:-4 5 6}; do
for i in 1 2; do
for v in head cur "$@"; do
  case $v in
    cur) L=$PWD/raytracing-project_amd/lib/librtamd.so ;;
    head) L=$PWD/raytracing-project_amd/lib/librtamd_head.so ;;
    *) L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so ;;
  esac
  RTAMD_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-100} --warmup 3 > gpurun_out/ab_${c}_${v}_$i.json 2> gpurun_out/ab_${c}_${v}_$i.err || { echo "bench $c $v failed"; tail gpurun_out/ab_${c}_${v}_$i.err; exit 1; }
  tail -1 gpurun_out/ab_${c}_${v}_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c $v', 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'])"
done; done; done
