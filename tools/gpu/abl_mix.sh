# Dynamic instruction mix per wave of the config-${CFG:-4} trace kernel for the product library
# and each ablation build lib/exp/librtamd_<v>.so (diagnostic builds, wrong images): two PMC passes
# each (every VALU class counter + SALU / LDS), "other" = VALU minus the classed ones (moves,
# selects, compares, lane ops).  Usage (GPU box): VARIANTS="abl1 abl2" bash tools/gpu/abl_mix.sh TAG
set -o pipefail
export TMPDIR=/tmp
T=${1:-ablmix}
CFG=${CFG:-4}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
for v in base ${VARIANTS}; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/raytracing-project_amd/lib/librtamd.so; else L=$GRAFT_REPO_ROOT/raytracing-project_amd/lib/exp/librtamd_$v.so; fi
  i=0
  for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32" \
             "SQ_WAVES SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS"; do
    i=$((i+1))
    RTAMD_LIB=$L timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/${v}_p$i -o pmc -- python3 tools/one_frame.py --config $CFG --frames 1 > $OUT/${v}_p$i.log 2>&1 || { echo "$v pass $i failed"; tail -5 $OUT/${v}_p$i.log; exit 1; }
  done
  python3 - $OUT $v <<'PY'
import csv, glob, os, sys, collections
out, v = sys.argv[1], sys.argv[2]
tot = collections.Counter()
for i in (1, 2):
    for f in glob.glob(os.path.join(out, f"{v}_p{i}", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if "k_std" not in row.get("Kernel_Name", "") and "k_paper_primary" not in row.get("Kernel_Name", ""):
                continue
            name = row["Counter_Name"]
            if name == "SQ_WAVES" and i == 2:
                continue
            tot[name] += float(row["Counter_Value"])
w = tot["SQ_WAVES"] or 1.0
g = lambda k: tot.get("SQ_INSTS_VALU_" + k, 0.0) / w
f64 = g("ADD_F64") + g("MUL_F64") + g("FMA_F64") + g("TRANS_F64")
f32 = g("ADD_F32") + g("MUL_F32") + g("FMA_F32") + g("TRANS_F32")
intg = g("INT32") + g("INT64")
cvt = g("CVT")
valu = tot["SQ_INSTS_VALU"] / w
print(f"{v:8s} VALU {valu:7.1f}  f64 {f64:7.1f}  f32 {f32:6.1f}  int {intg:6.1f}  cvt {cvt:5.1f}  other {valu - f64 - f32 - intg - cvt:7.1f}  SALU {tot['SQ_INSTS_SALU'] / w:7.1f}  LDS {tot['SQ_INSTS_LDS'] / w:5.1f}  waves {w:.0f}")
PY
done
