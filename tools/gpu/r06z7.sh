# Single-range jitter fill with no segment-list upload, and the rows list kept on the device across frames with the
# same rows: jitter / distributed tests, the parity subset, then base (the r06g build) vs cur, configs 4 3 2 6.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_jitter_rows.py tests/test_gpu_dist.py tests/test_gpu_dist_threads.py tests/test_gpu_runtime.py -x -q --timeout 200 --timeout-method thread > gpurun_out/z7_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/z7_tests.log; exit 1; }
tail -1 gpurun_out/z7_tests.log
CFGS="4 3 2 6" bash tools/gpu/ab_lib.sh base
