# Instruction-mix and instruction-cache PMC passes over tools/one_frame.py (one group per pass, nothing else enabled).
# Usage (GPU box): bash tools/gpu/pmc_detail.sh [config]
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-4}
OUT=gpurun_out/pmc_detail_$CFG
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_IFETCH SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM" \
           "SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE SQC_ICACHE_REQ"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/one_frame.py --config $CFG --frames 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > /dev/null && python3 - $CFG <<'PY'
import json
d = json.load(open(f"gpurun_out/pmc_detail_{__import__('sys').argv[1]}/summary.json"))
for k, m in d.items():
    if "k_std" not in k and "k_paper" not in k:
        continue
    w = m.get("SQ_WAVES", 1.0)
    print(k)
    for c, v in sorted(m.items()):
        if c.endswith("_per_wave"):
            continue
        print(f"  {c:30s} {v:14.4g}  {v / w:10.2f} /wave")
PY
