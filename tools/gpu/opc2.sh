set -o pipefail
export TMPDIR=/tmp
for v in cur ${LIBS:-nomask}; do
  if [ $v = cur ]; then L=$PWD/raytracing-project_amd/lib/librtamd.so; else L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so; fi
  echo "== $v"
  RTAMD_LIB=$L timeout -k 10 120 python tools/opcounts.py ${CFG:-4} 2>/dev/null | grep -v amdgpu.ids || { echo "$v failed"; exit 1; }
  RTAMD_LIB=$L ABLATE_QUICK=1 timeout -k 10 120 python tools/ablate.py ${CFG:-4} 2>&1 | grep -v amdgpu.ids || { echo "$v failed"; exit 1; }
done
