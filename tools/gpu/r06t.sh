# A/B on the plain kernels: 5 waves/SIMD (w5) and the lead-object path flipped (lflip: on in the recursion
# kernel, off in the paper kernel), configs 6 5 3 2.
set -o pipefail
export TMPDIR=/tmp
CFGS="6 5 3 2" bash tools/gpu/ab_lib.sh w5 lflip
