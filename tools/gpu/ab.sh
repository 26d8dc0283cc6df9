set -o pipefail
export TMPDIR=/tmp
for i in 1 2; do
RTAMD_LIB=$PWD/tools/ab/librtamd_head.so timeout -k 10 300 python tools/sim_ranks.py --worlds 1,8 > gpurun_out/ab_head_$i.log 2>&1 || { echo sim failed; tail gpurun_out/ab_head_$i.log; exit 1; }
timeout -k 10 300 python tools/sim_ranks.py --worlds 1,8 > gpurun_out/ab_new_$i.log 2>&1 || { echo sim failed; tail gpurun_out/ab_new_$i.log; exit 1; }
done
grep -h world gpurun_out/ab_head_*.log; echo; grep -h world gpurun_out/ab_new_*.log
