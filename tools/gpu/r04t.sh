# HIP runtime API + kernel trace of config 5's simulated ranks (world 8): where a rank's host time goes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04t}
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}_tr -o run -- python3 tools/sim_ranks.py --config 5 --worlds 8 --reps 3 > gpurun_out/${T}_sim.jsonl 2> gpurun_out/${T}_sim.err || { echo "trace failed"; tail gpurun_out/${T}_sim.err; exit 1; }
ls -R gpurun_out/${T}_tr | head -20
