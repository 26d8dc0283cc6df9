# Round-4: kernel trace of every simulated rank of config 5 (world 8) and config 4 (world 8) through the product path.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04i}
for c in 5 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${T}_tr$c -o run -- python3 tools/sim_ranks.py --config $c --worlds 1,8 --reps 2 > gpurun_out/${T}_sim$c.jsonl 2> gpurun_out/${T}_sim$c.err || { echo "trace $c failed"; tail gpurun_out/${T}_sim$c.err; exit 1; }
  f=$(find gpurun_out/${T}_tr$c -name '*kernel_trace.csv' | head -1)
  python3 tools/rank_trace.py $f 150 > gpurun_out/${T}_ranks$c.txt
  cat gpurun_out/${T}_ranks$c.txt | tail -30
done
