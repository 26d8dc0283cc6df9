# Row-walking paper finish (RT_FINISH_WALK rows per wave: fw8 / fw16 / fw32) against the block-of-rows finish (cur):
# the parity subset on fw16, then config-5 bench frames.
set -o pipefail
export TMPDIR=/tmp
RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_fw16.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullres_parity.py tests/test_gpu_dist_threads.py tests/test_gpu_crowd.py -x -q --timeout 200 --timeout-method thread > gpurun_out/fw_tests.log 2>&1 || { echo "fw16 tests failed"; tail -40 gpurun_out/fw_tests.log; exit 1; }
tail -1 gpurun_out/fw_tests.log
CFGS="5" bash tools/gpu/ab_lib.sh fw8 fw16 fw32
