# Wave BVH: its GPU tests (+ the parity / recursion suites whose scenes it can
# touch), then the perf comparison with and without the BVH and a config-4
# timing.  Usage (GPU box): bash tools/gpu/bvh.sh
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_bvh.py tests/test_bvh.py tests/test_gpu_parity.py tests/test_gpu_recursion.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bvh_tests.log 2>&1 || { echo "tests failed"; grep -E "^FAILED|Error|assert" gpurun_out/bvh_tests.log | head -20; tail -20 gpurun_out/bvh_tests.log; exit 1; }
tail -1 gpurun_out/bvh_tests.log
timeout -k 10 300 python tools/bvh_perf.py > gpurun_out/bvh_perf.txt 2>&1 || { echo "perf failed"; tail gpurun_out/bvh_perf.txt; exit 1; }
grep -v amdgpu.ids gpurun_out/bvh_perf.txt
for c in 4 5 6; do ABLATE_QUICK=1 timeout -k 10 120 python tools/ablate.py $c 2>&1 | grep -v amdgpu.ids || exit 1; done
