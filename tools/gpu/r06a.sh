# Round 6 first call: the changed distributed-protocol tests, then every config's bench line.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_threads.py tests/test_bench_launch.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r06a_dist.log 2>&1 || { echo "dist tests failed"; tail -30 gpurun_out/r06a_dist.log; exit 1; }
tail -2 gpurun_out/r06a_dist.log
STEPS=50 bash tools/gpu/configs.sh
