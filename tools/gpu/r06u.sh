# Check of the tuned plain kernels (parity subset, configs 3 6 against the round-6 start build), then the wave-cull
# threshold again on the plain kernels (RT_WV_MIN=3 / 1: configs 3 and 2 on the wave-culling kernel).
set -o pipefail
export TMPDIR=/tmp
CFGS="3 6" bash tools/gpu/ab_lib.sh || exit 1
CFGS="3 2" bash tools/gpu/ab_env.sh "RT_WV_MIN=3" "RT_WV_MIN=1"
