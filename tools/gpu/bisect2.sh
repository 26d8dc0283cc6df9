set -o pipefail
export TMPDIR=/tmp
run() { timeout -k 10 300 python -u -m pytest tests/test_gpu_jitter_rows.py -x -q --timeout 120 --timeout-method thread "$@" > gpurun_out/bisect2.log 2>&1; echo "[$RTAMD_LIB] $* rc=$? $(tail -1 gpurun_out/bisect2.log)"; }
RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_head.so run
RTAMD_LIB= run -k "jitter_stream or table_path"
RTAMD_LIB= run -k "row_subset_matches"
RTAMD_LIB= run -k "unordered"
RTAMD_LIB= run -k "two_streams"
