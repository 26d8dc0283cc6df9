# A/B: the per-lane leaf-ball shadow test compiled in (cur) or out (lib/exp/librtamd_nolane.so), configs 6 5 4.
set -o pipefail
export TMPDIR=/tmp
CFGS="6 5 4" bash tools/gpu/ab_lib.sh nolane
