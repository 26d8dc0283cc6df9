set -o pipefail
export TMPDIR=/tmp
L=$PWD/raytracing-project_amd/lib/exp/librtamd_${1:-prof}.so
for c in ${CFGS:-4 3}; do
  RTAMD_LIB=$L timeout -k 10 120 python tools/phase_prof.py $c 2>&1 | grep -v amdgpu.ids || { echo "phase $c failed"; exit 1; }
done
