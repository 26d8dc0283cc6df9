# Round-6 final evidence, part 1 (committed tree): full GPU suite, smoke, the default bench line (PMC traffic, CPU
# baseline, CLI leg), rocprofv3 kernel statistics of the bench, and the multi-GPU projections of configs 4 and 5.
# Usage (GPU box): TAG=r06f bash tools/gpu/r06_final2.sh      (part 2: TAG=r06f bash tools/gpu/r06_evidence.sh)
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06f}
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.log 2>&1 || { echo smoke failed; cat gpurun_out/${T}_smoke.log; exit 1; }
tail -1 gpurun_out/${T}_smoke.log
timeout -k 10 600 python bench.py > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
tail -1 gpurun_out/${T}_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- python bench.py --steps 50 --no-pmc --no-cpu --no-cli --fp32-steps 0 > gpurun_out/${T}_prof_bench.json 2>gpurun_out/${T}_prof.err || { echo prof failed; tail gpurun_out/${T}_prof.err; exit 1; }
find gpurun_out/${T}_prof -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats.csv
head -6 gpurun_out/${T}_kernel_stats.csv
timeout -k 10 600 python tools/sim_ranks.py --config 4 --worlds 1,2,4,8 > gpurun_out/${T}_sim_ranks.jsonl 2> gpurun_out/${T}_sim.err || { echo "sim 4 failed"; tail gpurun_out/${T}_sim.err; exit 1; }
timeout -k 10 600 python tools/sim_ranks.py --config 5 --worlds 1,2,4,8 >> gpurun_out/${T}_sim_ranks.jsonl 2>> gpurun_out/${T}_sim.err || { echo "sim 5 failed"; tail gpurun_out/${T}_sim.err; exit 1; }
python3 -c "
import json
for l in open('gpurun_out/${T}_sim_ranks.jsonl'):
    d=json.loads(l); print('cfg', d['config'], 'world', d['world'], 'max_wall', d['max_rank_wall_ms'], 'kmax', d['max_rank_kernel_ms'], 'x64', d['projected_speedup_64GBs'], 'x153', d['projected_speedup_153GBs'])"
