# Time config 4 (ABLATE_QUICK) with each experimental library in lib/exp (and the in-tree one as "cur").
# Usage (GPU box): bash tools/gpu/ablate_libs.sh name1 name2 ...
set -o pipefail
export TMPDIR=/tmp
for v in cur "$@"; do
  if [ $v = cur ]; then L=$PWD/raytracing-project_amd/lib/librtamd.so; else L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so; fi
  echo "== $v"
  RTAMD_LIB=$L ABLATE_QUICK=${ABLATE_QUICK-1} timeout -k 10 120 python tools/ablate.py ${ABLATE_CFG:-4} 2>&1 | grep -v amdgpu.ids || { echo "$v failed"; exit 1; }
done
