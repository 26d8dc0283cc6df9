# SQ counters of the trace kernel on config-4 sub-scenes (GPU box, diagnostic).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/vpmc
mkdir -p $OUT
for v in ${VARIANTS:-nolights_half nolights_nounion nolights full}; do
  timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU \
    --output-format csv -d $OUT/$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/render_variant.py $v > $OUT/$v.log 2>&1 || { echo "$v failed"; exit 1; }
done
echo done
