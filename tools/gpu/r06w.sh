# A/B: LDS light cache of 4 lights (lc4: 32 KiB per workgroup, 5 workgroups per CU for the plain lean kernel at
# 5 waves/SIMD) and of 3 lights with the plain lean kernel at 6 waves (lc3w6), configs 3 2 4.
set -o pipefail
export TMPDIR=/tmp
CFGS="3 2 4" bash tools/gpu/ab_lib.sh lc4 lc3w6
