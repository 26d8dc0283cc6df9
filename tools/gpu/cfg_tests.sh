set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
bash tools/gpu/configs.sh
timeout -k 10 300 python tools/sim_ranks.py --worlds 1,2,4,8 > gpurun_out/sim.log 2>&1 || { echo sim failed; tail gpurun_out/sim.log; exit 1; }
grep world gpurun_out/sim.log
