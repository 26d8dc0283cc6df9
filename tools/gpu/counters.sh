set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters_list.txt 2>&1 || { echo list failed; tail gpurun_out/counters_list.txt; exit 1; }
grep -oE "(SQ|TCP|TCC|TA|TD|SPI|GRBM)_[A-Z0-9_]+" gpurun_out/counters_list.txt | sort -u | tr '\n' ' ' | head -c 20000
