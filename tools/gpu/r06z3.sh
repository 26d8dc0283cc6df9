# One-wave standard workgroups (product now) against 4-wave ones (wpb4), configs 3 2 4 6, plain lean at 4 waves;
# and one-wave paper workgroups (pwpb1), config 5; then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
CFGS="3 2 4 6 5" bash tools/gpu/ab_lib.sh wpb4 pwpb1 || exit 1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
