set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_sim -o sim -- python tools/sim_ranks.py --worlds 8 --reps 2 > gpurun_out/prof_sim.log 2>&1 || { echo prof failed; tail gpurun_out/prof_sim.log; exit 1; }
cat gpurun_out/prof_sim/*/sim_kernel_stats.csv 2>/dev/null || find gpurun_out/prof_sim -name "*kernel_stats.csv" -exec cat {} \;
