# Round-6 per-config evidence on one tree: for configs 2-6, the bench line, the rocprofv3 kernel
# statistics of a short bench run, and the PMC instruction mix (three counter passes, per wave).
# Usage (GPU box): TAG=r06z CFGS="2 3 4 5 6" bash tools/gpu/r06_evidence.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06z}
for c in ${CFGS:-2 3 4 5 6}; do
  timeout -k 10 300 python bench.py --config $c --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps ${STEPS:-100} --warmup 3 > gpurun_out/${T}_bench_c$c.json 2> gpurun_out/${T}_bench_c$c.err || { echo "bench $c failed"; tail gpurun_out/${T}_bench_c$c.err; exit 1; }
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof_c$c -o run --output-format csv -- python bench.py --config $c --steps 30 --warmup 2 --no-pmc --no-cpu --no-cli --fp32-steps 0 > gpurun_out/${T}_prof_c$c.log 2>&1 || { echo "prof $c failed"; tail gpurun_out/${T}_prof_c$c.log; exit 1; }
  CFG=$c timeout -k 10 600 bash tools/gpu/pmc_mix_cfg.sh > gpurun_out/${T}_pmc_c$c.txt 2>&1 || { echo "pmc $c failed"; tail gpurun_out/${T}_pmc_c$c.txt; exit 1; }
  echo "config $c done"
done
