# Dynamic-LDS shading pool (per-wave regions) + paper root shed 45: full GPU suite, then the standard-mode workgroup
# size A/B (RT_STD_WPB 4 = product, 1, 2: one / two waves per workgroup), configs 4 3 6.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { echo "tests failed"; tail -60 gpurun_out/gpu_tests.log; exit 1; }
tail -3 gpurun_out/gpu_tests.log
CFGS="4 3 6" bash tools/gpu/ab_lib.sh wpb1 wpb2
