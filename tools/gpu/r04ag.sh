# Round-4: agreement issued after chunk 0's launch: dist tests + projections.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04ag}
timeout -k 10 400 python -u -m pytest tests/test_gpu_dist.py tests/test_gpu_jitter_rows.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -1 gpurun_out/${T}_tests.log
TAG=${T} timeout -k 10 500 bash tools/gpu/r04sim.sh
