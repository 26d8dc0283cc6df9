#!/bin/bash
# PMC passes for the bench workload (one counter group per pass; no tracing
# domains combined with --pmc).  Output under gpurun_out/pmc_*.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out}
ARGS=${ARGS:---steps 1 --warmup 1 --no-cpu}
rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$i -o pmc -- python bench.py $ARGS > $OUT/pmc_$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
echo done
