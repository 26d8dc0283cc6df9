# A/B: wave-uniform bundle parameters moved to SGPRs in the standard kernels and kept in VGPRs in the paper kernels
# (uo: RT_STD_UO=true, RT_PAPER_UO=false; the product has the opposite), configs 4 6 5.
set -o pipefail
export TMPDIR=/tmp
CFGS="4 6 5" bash tools/gpu/ab_lib.sh uo
