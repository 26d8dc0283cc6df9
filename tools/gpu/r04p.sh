# Kernel trace of config 5's simulated ranks (world 8) through the product rank path (shared streams).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04p}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr5 -o run -- python3 tools/sim_ranks.py --config 5 --worlds 8 --reps 3 > gpurun_out/${T}_sim5.jsonl 2> gpurun_out/${T}_sim5.err || { echo "trace failed"; tail gpurun_out/${T}_sim5.err; exit 1; }
cat gpurun_out/${T}_sim5.jsonl
