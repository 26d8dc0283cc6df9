# First-op probe, then fresh phase timers and event counts of configs 4 and 3 (diagnostic builds in lib/exp).
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/first_op.sh > gpurun_out/r06d_first_op.txt 2>&1 || { echo probe failed; cat gpurun_out/r06d_first_op.txt; exit 1; }
cat gpurun_out/r06d_first_op.txt
CFGS="4 3" bash tools/gpu/phase.sh prof > gpurun_out/r06e_phase.txt 2>&1 || { echo phase failed; tail gpurun_out/r06e_phase.txt; exit 1; }
cat gpurun_out/r06e_phase.txt
for c in 4 3; do RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_ev.so timeout -k 10 120 python tools/event_prof.py $c > gpurun_out/r06e_events_$c.txt 2>&1 || { echo events failed; tail gpurun_out/r06e_events_$c.txt; exit 1; }; cat gpurun_out/r06e_events_$c.txt; done
