# Memory-side PMC passes over tools/one_frame.py (one group per pass): vector / scalar / LDS instruction counts, LDS waits and bank conflicts, scalar-cache and L1/L2 hit rates.
# Usage (GPU box): bash tools/gpu/pmc_mem.sh [config]
set -o pipefail
export TMPDIR=/tmp
CFG=${1:-4}
OUT=gpurun_out/pmc_mem_$CFG
rm -rf $OUT; mkdir -p $OUT
i=0
for grp in "SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT" \
           "SQC_DCACHE_HITS SQC_DCACHE_MISSES SQC_DCACHE_REQ" \
           "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o pmc -- python3 tools/one_frame.py --config $CFG --frames 2 > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 tools/pmc_summary.py $OUT > /dev/null && python3 - $CFG <<'PY'
import json
d = json.load(open(f"gpurun_out/pmc_mem_{__import__('sys').argv[1]}/summary.json"))
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
