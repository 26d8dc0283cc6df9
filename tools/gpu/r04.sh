# Round-4 evidence run on the committed tree: full GPU suite, smoke, default bench line,
# rocprofv3 kernel-trace summary of a short bench, per-config kernel traces and PMC
# instruction mixes of the trace kernels of configs 4, 5 and 6.
# Usage (GPU box): TAG=r04n bash tools/gpu/r04.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04n}

TAG=$T timeout -k 10 1000 bash tools/gpu/r03.sh || exit 1
for c in 5 6; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof$c -o run --output-format csv -- python3 tools/one_frame.py --config $c --frames 20 > gpurun_out/${T}_prof$c.log 2>&1 || { echo "prof $c failed"; exit 1; }
  find gpurun_out/${T}_prof$c -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats_cfg$c.csv
done
for c in 4 5 6; do
  timeout -k 10 400 bash tools/gpu/pmc_detail.sh $c > gpurun_out/${T}_pmc_detail_cfg$c.txt 2>&1 || { echo "pmc $c failed"; exit 1; }
done
echo done
