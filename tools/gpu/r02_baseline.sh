# Round-2 baseline: ablations of config 4 and per-config bench lines (diagnostic).
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/ablate.py 4 > gpurun_out/ablate_c4.log 2>&1 || { echo "ablate failed"; tail gpurun_out/ablate_c4.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ablate_c4.log
bash tools/gpu/configs.sh
