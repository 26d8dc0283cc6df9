# Round-4: distributed-frame failure handling tests + config-5 rank-share sweep
# (strip height x chunk count) on one GPU.  Usage: TAG=r04b bash tools/gpu/r04b.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04b}
timeout -k 10 300 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_cli.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_dist_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_dist_tests.log; exit 1; }
tail -3 gpurun_out/${T}_dist_tests.log
: > gpurun_out/${T}_sim5_sweep.jsonl
for ch in 4 1; do
  for s in 30 62 126; do
    timeout -k 10 200 python3 tools/sim_ranks.py --config 5 --worlds 1,8 --reps 3 --strip $s --chunks $ch >> gpurun_out/${T}_sim5_sweep.jsonl 2> gpurun_out/${T}_sim5.err || { echo "sim failed"; tail gpurun_out/${T}_sim5.err; exit 1; }
  done
done
cat gpurun_out/${T}_sim5_sweep.jsonl
