# PMC instruction mix (per wave) of config ${CFG:-4}'s trace kernels (rocprofv3 --pmc, one group per pass).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_mix_c${CFG:-4}
mkdir -p $OUT
i=0
for grp in "SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_INT32" \
           "SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FLOPS_FP64 SQ_INSTS_VALU_FLOPS_FP32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INST_CYCLES_SALU" \
           "SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_BRANCH" \
           "SQ_WAVES SQ_WAIT_ANY SQ_INSTS_LDS"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python bench.py --config ${CFG:-4} --steps 1 --warmup 0 --no-cpu --no-pmc --no-cli --fp32-steps 0 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail $OUT/p$i.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
per = collections.defaultdict(lambda: collections.defaultdict(list))
import os
for f in glob.glob("gpurun_out/pmc_mix_c%s/p*/**/*counter_collection.csv" % os.environ.get("CFG", "4"), recursive=True):
    for r in csv.DictReader(open(f)):
        if "k_std" in r["Kernel_Name"] or "k_paper" in r["Kernel_Name"]:
            per[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in per.items():
    print(k)
    waves = sum(cs["SQ_WAVES"]) / len(cs["SQ_WAVES"]) if cs.get("SQ_WAVES") else None
    for c, v in sorted(cs.items()):
        avg = sum(v) / len(v)
        pw = f"  per wave {avg / waves:.5g}" if waves else ""
        print(f"  {c:28s} {avg:.6g}  (n={len(v)}){pw}")
PY
