# Config 4 after the per-lane leaf test: phase timers, event counts, PMC instruction mix; config 3 PMC mix.
set -o pipefail
export TMPDIR=/tmp
CFGS="4" bash tools/gpu/phase.sh prof > gpurun_out/r06n_phase.txt 2>&1 || { echo phase failed; tail gpurun_out/r06n_phase.txt; exit 1; }
cat gpurun_out/r06n_phase.txt
RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_ev.so timeout -k 10 120 python tools/event_prof.py 4 > gpurun_out/r06n_events_4.txt 2>&1 || { echo events failed; tail gpurun_out/r06n_events_4.txt; exit 1; }
cat gpurun_out/r06n_events_4.txt
CFG=4 timeout -k 10 600 bash tools/gpu/pmc_mix_cfg.sh > gpurun_out/r06n_pmc_c4.txt 2>&1 || { echo "pmc 4 failed"; tail gpurun_out/r06n_pmc_c4.txt; exit 1; }
cat gpurun_out/r06n_pmc_c4.txt
CFG=3 timeout -k 10 600 bash tools/gpu/pmc_mix_cfg.sh > gpurun_out/r06n_pmc_c3.txt 2>&1 || { echo "pmc 3 failed"; tail gpurun_out/r06n_pmc_c3.txt; exit 1; }
cat gpurun_out/r06n_pmc_c3.txt
