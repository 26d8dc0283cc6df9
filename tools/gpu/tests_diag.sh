# Full GPU suite (one process) + phase / wave-event diagnostics of the trace kernel for $CFGS.
# Usage (GPU box): TAG=r03d CFGS="6 4" bash tools/gpu/tests_diag.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r03}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/${T}_gpu_tests.log | head -30; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -1 gpurun_out/${T}_gpu_tests.log
for c in ${CFGS:-4}; do
  RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_prof.so timeout -k 10 200 python tools/phase_prof.py $c 2>&1 | grep -v amdgpu.ids || { echo "phase $c failed"; exit 1; }
  RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_ev.so timeout -k 10 200 python tools/event_prof.py $c 2>&1 | grep -v amdgpu.ids || { echo "events $c failed"; exit 1; }
done
