# Full GPU suite on the kernel-copy upload build, then the CLI timing and its API/kernel trace.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06g_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06g_gpu_tests.log; exit 1; }
tail -2 gpurun_out/r06g_gpu_tests.log
TAG=r06g bash tools/gpu/cli_prof.sh
