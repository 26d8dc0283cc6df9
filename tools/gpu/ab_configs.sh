# Kernel time of configs 2-5 (their own mode) for the in-tree library and each lib/exp/librtamd_<name>.so.
# Usage (GPU box): bash tools/gpu/ab_configs.sh name1 ...
set -o pipefail
for c in 2 3 4 5; do echo "## config $c"; ABLATE_CFG=$c bash tools/gpu/ablate_libs.sh "$@" || exit 1; done
