# A/B of library builds on the many-object scenes (tools/bvh_perf.py): head, cur and lib/exp/librtamd_<name>.so.
# Usage (GPU box): bash tools/gpu/ab_bvh.sh [name ...]
set -o pipefail
export TMPDIR=/tmp
for v in head cur "$@"; do
  case $v in
    cur) L=$PWD/raytracing-project_amd/lib/librtamd.so ;;
    head) L=$PWD/raytracing-project_amd/lib/librtamd_head.so ;;
    *) L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so ;;
  esac
  echo "== $v"
  RTAMD_LIB=$L timeout -k 10 300 python tools/bvh_perf.py 2>&1 | grep -v amdgpu.ids || exit 1
done
