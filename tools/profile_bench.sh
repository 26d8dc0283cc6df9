#!/bin/bash
# Profile the bench workload on the GPU box: kernel trace + stats, then one
# PMC pass per counter group (never combined with tracing domains).
# Usage (from the repo root): TAG=r01 bash tools/profile_bench.sh
set -o pipefail
export TMPDIR=/tmp
TAG=${TAG:-r01}
OUT=gpurun_out/prof_$TAG
ARGS=${ARGS:---steps 3 --warmup 1 --no-cpu --fp32-steps 0}
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o bench -- python bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace pass failed"; exit 1; }
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_$i -o pmc -- python bench.py --steps 1 --warmup 1 --no-cpu --fp32-steps 0 > $OUT/pmc_$i.log 2>&1 || { echo "pmc pass $i failed"; exit 1; }
done
python tools/summarize_profile.py $OUT $OUT/summary $TAG  # copy into profiles/ locally after the call
