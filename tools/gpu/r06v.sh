# A/B: jitter draws as non-temporal stores (lib/exp/librtamd_jnt.so, -DRT_JIT_NT in mt_jump.hip), configs 4 3.
set -o pipefail
export TMPDIR=/tmp
CFGS="4 3" bash tools/gpu/ab_lib.sh jnt
