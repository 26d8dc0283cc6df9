# Phase timers and event counts of configs 5 and 6 (diagnostic builds in lib/exp), then the A/B of the
# capsule far end at the light (in-tree build) against -DRT_NO_CAP_LIGHT (lib/exp/librtamd_nocl.so).
set -o pipefail
export TMPDIR=/tmp
CFGS="5 6" bash tools/gpu/phase.sh prof > gpurun_out/r06o_phase.txt 2>&1 || { echo phase failed; tail gpurun_out/r06o_phase.txt; exit 1; }
cat gpurun_out/r06o_phase.txt
for c in 5 6; do RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_ev.so timeout -k 10 120 python tools/event_prof.py $c > gpurun_out/r06o_events_$c.txt 2>&1 || { echo events failed; tail gpurun_out/r06o_events_$c.txt; exit 1; }; cat gpurun_out/r06o_events_$c.txt; done
CFGS="4 5 6" bash tools/gpu/ab_lib.sh nocl
