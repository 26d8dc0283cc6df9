# Parity subset on the in-tree build (config 4 at full size with culling on and off included), then
# A/B of lib/librtamd_head.so, lib/exp/librtamd_<variants> and the in-tree lib on configs ${CFGS:-4 3 5}.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py tests/test_gpu_crowd.py tests/test_gpu_bvh.py tests/test_gpu_recursion.py tests/test_gpu_edges.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06i_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06i_tests.log; exit 1; }
tail -1 gpurun_out/r06i_tests.log
for c in ${CFGS:-4 3 5}; do
for i in 1 2; do
for v in head ${VARIANTS:-nolane} cur; do
  case $v in
    cur) L=$PWD/raytracing-project_amd/lib/librtamd.so ;;
    head) L=$PWD/raytracing-project_amd/lib/librtamd_head.so ;;
    *) L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so ;;
  esac
  RTAMD_LIB=$L timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-100} --warmup 3 > gpurun_out/ab_${c}_${v}_$i.json 2> gpurun_out/ab_${c}_${v}_$i.err || { echo "bench $c $v failed"; tail gpurun_out/ab_${c}_${v}_$i.err; exit 1; }
  tail -1 gpurun_out/ab_${c}_${v}_$i.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c $v', 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'], 'exec_frac', d['roofline']['executed_frac'])"
done; done; done
