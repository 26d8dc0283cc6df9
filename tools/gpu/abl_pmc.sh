# Ablation A/B of the config-4 trace kernel (diagnostic builds, wrong images):
# kernel time (tools/ablate.py, ABLATE_QUICK) and SQ instruction counts per wave
# (rocprofv3 --pmc over tools/one_frame.py) for the product library and each
# lib/exp/librtamd_<v>.so.   Usage (GPU box): VARIANTS="abl1 abl2" bash tools/gpu/abl_pmc.sh TAG
export TMPDIR=/tmp
T=${1:-abl}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
for v in base ${VARIANTS}; do
  if [ $v = base ]; then L=$GRAFT_REPO_ROOT/raytracing-project_amd/lib/librtamd.so; else L=$GRAFT_REPO_ROOT/raytracing-project_amd/lib/exp/librtamd_$v.so; fi
  RTAMD_LIB=$L ABLATE_QUICK=1 timeout -k 10 90 python3 tools/ablate.py 4 > $OUT/$v.time 2>&1 || { echo "$v time failed"; cat $OUT/$v.time; exit 1; }
  RTAMD_LIB=$L timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64 \
    --output-format csv -d $OUT/$v -o pmc -- python3 tools/one_frame.py --config 4 --frames 1 > $OUT/$v.log 2>&1 || { echo "$v pmc failed"; tail $OUT/$v.log; exit 1; }
  python3 tools/pmc_summary.py $OUT/$v > /dev/null
  python3 - $OUT/$v <<'PY'
import json, sys, os
d = json.load(open(os.path.join(sys.argv[1], "summary.json")))
t = open(sys.argv[1] + ".time").read().strip().splitlines()[-1]
for k, m in d.items():
    if "k_std" in k:
        w = m["SQ_WAVES"]
        f64 = sum(m.get(c, 0) for c in ("SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_TRANS_F64")) / w
        print(f"{os.path.basename(sys.argv[1]):10s} VALU/wave {m['SQ_INSTS_VALU']/w:8.1f}  f64 {f64:7.1f}  SALU/wave {m['SQ_INSTS_SALU']/w:8.1f}  activeVALU/wave {m['SQ_ACTIVE_INST_VALU']/w:8.1f} | {t}")
PY
done
timeout -k 10 120 python3 tools/cli_time.py 4 > $OUT/cli.txt 2>&1 || echo "cli timing failed"
cat $OUT/cli.txt
