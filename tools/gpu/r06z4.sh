# A/B with one-wave workgroups: the standard wave's pixel tile (RT_STD_TW: product 2 = 2x4 pixels; tw4 = 4x2; tw1 = 1x8),
# configs 4 6 3.
set -o pipefail
export TMPDIR=/tmp
CFGS="4 6 3" bash tools/gpu/ab_lib.sh tw4 tw1
