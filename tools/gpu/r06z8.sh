# Counter slots cleared by the frame-end reduction instead of a memset at frame start: full GPU suite (ray counts and
# op counts every test), then base (previous build) vs cur, configs 2 3 4.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
CFGS="2 3 4" bash tools/gpu/ab_lib.sh base
