# Plain kernels: A/B against RT_PLAIN=0 (the general variants) on configs 6 5 3 2, then the full GPU suite.
set -o pipefail
export TMPDIR=/tmp
CFGS="6 5 3 2" bash tools/gpu/ab_env.sh "RT_PLAIN=0" || exit 1
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
