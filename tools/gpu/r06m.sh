# Jitter-table segment length K=8 (lib/exp8) vs the product's 16, and root shed A/B, in the multi-GPU projection.
set -o pipefail
export TMPDIR=/tmp
K8=$PWD/raytracing-project_amd/lib/exp8/librtamd_k8.so
RTAMD_LIB=$K8 timeout -k 10 600 python -u -m pytest tests/test_gpu_jitter_rows.py tests/test_gpu_fullres_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r06m_k8_tests.log 2>&1 || { echo "k8 tests failed"; tail -30 gpurun_out/r06m_k8_tests.log; exit 1; }
tail -1 gpurun_out/r06m_k8_tests.log
OUT=gpurun_out/r06m_sim.jsonl
: > $OUT
run() {   # label, then env assignments, then sim args
  local lab=$1; shift
  env "$@" timeout -k 10 300 python tools/sim_ranks.py $SIMARGS > gpurun_out/sim_tmp.jsonl 2> gpurun_out/sim_tmp.err || { echo "sim $lab failed"; tail gpurun_out/sim_tmp.err; exit 1; }
  python3 -c "import json; [print(json.dumps(dict(json.loads(l), ab='$lab'))) for l in open('gpurun_out/sim_tmp.jsonl') if l.startswith('{')]" >> $OUT
}
for i in 1 2; do
  SIMARGS="--config 4 --worlds 1,8" run k16 X=1
  SIMARGS="--config 4 --worlds 1,8" run k8 RTAMD_LIB=$K8
done
for s in 8 12 16; do SIMARGS="--config 4 --worlds 1,8" run shed_std=$s RT_ROOT_SHED_STD=$s; done
for s in 30 45 60; do SIMARGS="--config 5 --worlds 1,2,4,8" run shed_paper=$s RT_ROOT_SHED_PAPER=$s; done
python3 -c "
import json
for l in open('$OUT'):
    d=json.loads(l); print(d['ab'], 'cfg', d['config'], 'world', d['world'], 'max_wall', d['max_rank_wall_ms'], 'r0', d['rank0_wall_ms'], 'kmax', d['max_rank_kernel_ms'], 'x64', d['projected_speedup_64GBs'], 'x153', d['projected_speedup_153GBs'])"
