# A/B: kernels without the transform / CSG object code (lib/exp/librtamd_nocsg.so, -DRT_EXP_NOCSG; the
# scenes of configs 2, 3, 5, 6 have none) against the in-tree build.
set -o pipefail
export TMPDIR=/tmp
CFGS="6 5 3 2" bash tools/gpu/ab_lib.sh nocsg
