# Round-5 check: full GPU suite, per-config bench lines (CFGS, default "4 5"),
# rocprofv3 kernel stats of config 5 (paper) frames.
# Usage (GPU box): TAG=r05b [CFGS="4 5"] bash tools/gpu/r05.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05x}
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|error" gpurun_out/${T}_gpu_tests.log | head -40; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
CFGS=${CFGS:-4 5} STEPS=${STEPS:-30} timeout -k 10 600 bash tools/gpu/configs.sh || exit 1
if [ -n "$PROF5" ]; then
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_prof5 -o run --output-format csv -- python3 tools/one_frame.py --config 5 --frames 20 > gpurun_out/${T}_prof5.log 2>&1 || { echo "prof 5 failed"; exit 1; }
  find gpurun_out/${T}_prof5 -name '*kernel_stats.csv' | head -1 | xargs -I{} cp {} gpurun_out/${T}_kernel_stats_cfg5.csv
  head -6 gpurun_out/${T}_kernel_stats_cfg5.csv | cut -c1-200
fi
echo done
