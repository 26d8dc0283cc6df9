# quick check: parity subset + config-4 timing + phase breakdown (diagnostic)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py -x -q --timeout 200 --timeout-method thread ${PYTEST_K:+-k "$PYTEST_K"} > gpurun_out/check_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/check_tests.log; exit 1; }
tail -3 gpurun_out/check_tests.log
ABLATE_QUICK=1 timeout -k 10 120 python tools/ablate.py 4 2>&1 | grep -v amdgpu.ids || exit 1
CFGS=4 bash tools/gpu/phase.sh prof
