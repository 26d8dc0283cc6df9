# Round-4: last chunk on the frame's stream + parallel counter reduction; dist tests, sim sweep, bench, API trace.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04v}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_jitter_rows.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo "bench failed"; tail gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'])"
: > gpurun_out/${T}_sim.jsonl
for c in 5 4; do
  timeout -k 10 200 python3 tools/sim_ranks.py --config $c --worlds 1,2,4,8 --reps 10 >> gpurun_out/${T}_sim.jsonl 2> gpurun_out/${T}_sim.err || { echo "sim failed"; tail gpurun_out/${T}_sim.err; exit 1; }
done
python3 - <<PY
import json
for l in open("gpurun_out/${T}_sim.jsonl"):
    d = json.loads(l)
    print(d["config"], d["chunks"], d["world"], d["max_rank_wall_ms"], d["rank0_wall_ms"], d["min_rank_wall_ms"], d["last_chunk_place_ms"], d["frame_ms_153GBs"], d["projected_speedup_153GBs"], d["projected_speedup_64GBs"])
PY
timeout -k 10 300 rocprofv3 --kernel-trace --hip-runtime-trace --memory-copy-trace --output-format csv -d gpurun_out/${T}_tr -o run -- python3 tools/sim_ranks.py --config 5 --worlds 8 --reps 3 > gpurun_out/${T}_trsim.jsonl 2> gpurun_out/${T}_trsim.err || { echo "trace failed"; tail gpurun_out/${T}_trsim.err; exit 1; }
