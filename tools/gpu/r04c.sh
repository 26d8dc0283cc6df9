# Round-4: distributed-frame tests (paper codes, agreement, fault injection) +
# per-rank projections through the product's rank path for configs 4 and 5.
# Usage: TAG=r04c bash tools/gpu/r04c.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04c}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_cli.py tests/test_gpu_parity.py -m gpu -x -v -s --timeout 120 --timeout-method thread > gpurun_out/${T}_dist_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_dist_tests.log; exit 1; }
tail -3 gpurun_out/${T}_dist_tests.log
grep "timeout path" gpurun_out/${T}_dist_tests.log
: > gpurun_out/${T}_sim_ranks.jsonl
for c in 5 4; do
  timeout -k 10 300 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 5 >> gpurun_out/${T}_sim_ranks.jsonl 2> gpurun_out/${T}_sim.err || { echo "sim failed"; tail gpurun_out/${T}_sim.err; exit 1; }
done
cat gpurun_out/${T}_sim_ranks.jsonl
