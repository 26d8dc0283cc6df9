# Round-4: XCD-aware finish tiles: paper tests, config-5 kernel stats, HBM traffic passes.
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04xcd}
TAG=$T timeout -k 10 700 bash tools/gpu/r04x.sh || exit 1
TAG=${T}_hbm timeout -k 10 300 bash tools/gpu/r04hbm5.sh || exit 1
