# First-op probe; parity subset of the current build; CLI timing; phase timers + event counts (lib/exp diagnostics).
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/first_op.sh > gpurun_out/r06d_first_op.txt 2>&1 || { echo probe failed; cat gpurun_out/r06d_first_op.txt; exit 1; }
cat gpurun_out/r06d_first_op.txt
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_jitter_rows.py tests/test_gpu_cli.py tests/test_gpu_numerics.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r06f_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/r06f_tests.log; exit 1; }
tail -1 gpurun_out/r06f_tests.log
timeout -k 10 120 python3 tools/cli_time.py 4 > gpurun_out/r06f_cli_time.txt 2>&1 || { tail gpurun_out/r06f_cli_time.txt; exit 1; }
cat gpurun_out/r06f_cli_time.txt
CFGS="4 3" bash tools/gpu/phase.sh prof > gpurun_out/r06e_phase.txt 2>&1 || { echo phase failed; tail gpurun_out/r06e_phase.txt; exit 1; }
cat gpurun_out/r06e_phase.txt
for c in 4 3; do RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_ev.so timeout -k 10 120 python tools/event_prof.py $c > gpurun_out/r06e_events_$c.txt 2>&1 || { echo events failed; tail gpurun_out/r06e_events_$c.txt; exit 1; }; cat gpurun_out/r06e_events_$c.txt; done
