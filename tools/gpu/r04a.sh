# Round-4 first GPU pass: rocprofv3 kernel traces + instruction-mix PMC for the
# paper kernels (config 5) and the recursion kernel (config 6), config 5's
# 8-way rank share under the kernel trace, and a short bench on the new launcher.
# Usage (GPU box): TAG=r04a bash tools/gpu/r04a.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04a}
for c in 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof$c -o run --output-format csv -- python3 tools/one_frame.py --config $c --frames 20 > gpurun_out/${T}_prof$c.log 2>&1 || { echo "prof $c failed"; tail gpurun_out/${T}_prof$c.log; exit 1; }
  find gpurun_out/${T}_prof$c -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats_cfg$c.csv
  head -6 gpurun_out/${T}_kernel_stats_cfg$c.csv
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_profsim5 -o run --output-format csv -- python3 tools/sim_ranks.py --config 5 --worlds 1,8 --reps 3 > gpurun_out/${T}_sim5.jsonl 2> gpurun_out/${T}_sim5.err || { echo "sim5 failed"; tail gpurun_out/${T}_sim5.err; exit 1; }
find gpurun_out/${T}_profsim5 -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats_sim5.csv
cat gpurun_out/${T}_sim5.jsonl
for c in 5 6; do
  timeout -k 10 400 bash tools/gpu/pmc_detail.sh $c > gpurun_out/${T}_pmc_detail_cfg$c.txt 2>&1 || { echo "pmc $c failed"; tail gpurun_out/${T}_pmc_detail_cfg$c.txt; exit 1; }
done
timeout -k 10 300 python bench.py --steps 100 --no-cpu --no-pmc --no-cli > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
tail -c 600 gpurun_out/${T}_bench.json
