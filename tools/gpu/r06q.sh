# A/B of the lead-object path per query kind in the recursion / paper kernels (li0: closest-hit without it,
# ls0: shadow without it, l00: neither), configs 6 and 5; then config 5/6 phase timers (fixed chunk timing).
set -o pipefail
export TMPDIR=/tmp
CFGS="6 5" bash tools/gpu/ab_lib.sh li0 ls0 l00 || exit 1
CFGS="5 6" bash tools/gpu/phase.sh prof > gpurun_out/r06q_phase.txt 2>&1 || { echo phase failed; tail gpurun_out/r06q_phase.txt; exit 1; }
cat gpurun_out/r06q_phase.txt
