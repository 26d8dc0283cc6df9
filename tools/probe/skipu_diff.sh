set -o pipefail
export TMPDIR=/tmp
L=$PWD/raytracing-project_amd/lib/exp/librtamd_${1:-skipu}.so
timeout -k 10 120 python tools/probe/render_npy.py snorlax 0 gpurun_out/cur.npy 2>&1 | grep -v amdgpu || exit 1
RTAMD_LIB=$L timeout -k 10 120 python tools/probe/render_npy.py snorlax 0 gpurun_out/skipu.npy 2>&1 | grep -v amdgpu || exit 1
RTAMD_LIB=$L timeout -k 10 120 python tools/probe/render_npy.py snorlax 0 gpurun_out/skipu_nocull.npy 2 2>&1 | grep -v amdgpu || exit 1
python - <<'PY'
import numpy as np
a = np.load("gpurun_out/cur.npy"); b = np.load("gpurun_out/skipu.npy"); c = np.load("gpurun_out/skipu_nocull.npy")
d = np.abs(a - b).max(axis=2); ys, xs = np.nonzero(d)
print("diff px", len(ys), "max", d.max())
print(list(zip(ys[:30].tolist(), xs[:30].tolist())))
print("skipu nocull vs cur diff px", int((np.abs(a - c).max(axis=2) > 0).sum()))
PY
