# PMC passes (one counter group per pass, nothing else enabled) over
# tools/one_frame.py; per-wave summary of the trace kernel.  Usage: bash tools/gpu/pmc_frame.sh [config] [RTAMD_LIB]
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-4}
OUT=gpurun_out/pmc_frame
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE GRBM_COUNT" \
           "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/one_frame.py --config $CFG --frames 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT
