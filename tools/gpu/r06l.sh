# Parity subset; RT_LEAD A/B on configs 4 5 6; the multi-GPU projection A/B (chunk counts).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py tests/test_gpu_crowd.py tests/test_gpu_bvh.py tests/test_gpu_recursion.py tests/test_gpu_edges.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06l_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06l_tests.log; exit 1; }
tail -1 gpurun_out/r06l_tests.log
for c in 4 5 6; do
for i in 1 2; do
for v in 0 1; do
  RT_LEAD=$v timeout -k 10 200 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps 100 --warmup 3 > gpurun_out/abl_${c}_${v}_${i}.json 2> gpurun_out/abl_${c}_${v}_${i}.err || { echo "bench $c $v failed"; tail gpurun_out/abl_${c}_${v}_${i}.err; exit 1; }
  tail -1 gpurun_out/abl_${c}_${v}_${i}.json | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg $c lead=$v', 'frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'], 'value', d['value'])"
done; done; done
TAG=r06l bash tools/gpu/sim_ab.sh
