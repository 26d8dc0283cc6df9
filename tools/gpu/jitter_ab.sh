# Jitter-table A/B: parity of a variant library (jitter + multi-rank tests), then
# per-rank projections (config 4, 1 and 8 ranks) and the N=1 frame for the
# in-tree library and the variant.  Usage (GPU box): bash tools/gpu/jitter_ab.sh NAME
set -o pipefail
export TMPDIR=/tmp
L=$PWD/raytracing-project_amd/lib/exp/librtamd_$1.so
RTAMD_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_jitter_rows.py tests/test_gpu_dist.py -x -q --timeout 300 --timeout-method thread > gpurun_out/$1_tests.log 2>&1 || { echo "tests failed"; tail -20 gpurun_out/$1_tests.log; exit 1; }
tail -1 gpurun_out/$1_tests.log
for v in cur $1; do
  if [ $v = cur ]; then LL=; else LL=$L; fi
  echo "== $v"
  RTAMD_LIB=$LL timeout -k 10 300 python tools/sim_ranks.py --config ${CFG:-4} --worlds 1,8 --reps 3 > gpurun_out/$1_sim_$v.jsonl 2>/dev/null || { echo sim failed; exit 1; }
  python - gpurun_out/$1_sim_$v.jsonl <<'PY'
import json, sys
for l in open(sys.argv[1]):
    d = json.loads(l)
    print(d["world"], "wall", d["max_rank_wall_ms"], "rng", d["max_rank_rng_ms"], "kernel", d["max_rank_kernel_ms"],
          "proj", d["projected_speedup_64GBs"], d["projected_speedup_153GBs"])
PY
  RTAMD_LIB=$LL timeout -k 10 200 python bench.py --config ${CFG:-4} --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps 100 > gpurun_out/$1_bench_$v.json 2>/dev/null || { echo bench failed; exit 1; }
  python - gpurun_out/$1_bench_$v.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("frame", d["ms_per_step"], "kernel", d["roofline"]["kernel_ms"], "rng", d["wall_clock_ms"]["rng"], "first", d["first_frame_ms"])
PY
done
