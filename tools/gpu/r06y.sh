# Root shed of the paper partition with the plain paper kernel (config 5 projections at 8 ranks), chunks 2 and 3.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/shed.sh 30 45 55 62 || exit 1
RT_DIST_CHUNKS_PAPER=3 bash tools/gpu/shed.sh 30 45 55 62
