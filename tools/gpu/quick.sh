# Quick A/B: parity subset on the in-tree library, then config-4 (and 3, 5) kernel time for cur vs lib/exp variants.
# Usage (GPU box): bash tools/gpu/quick.sh name1 ...
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/quick_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/quick_tests.log; exit 1; }
tail -1 gpurun_out/quick_tests.log
for c in ${QCFGS:-4}; do echo "## config $c"; ABLATE_CFG=$c bash tools/gpu/ablate_libs.sh "$@" || exit 1; done
