# PC sampling of the config-N trace kernel (stochastic, cycles) with the line-table build
# lib/exp/librtamd_dbg.so; the samples CSV lands under gpurun_out/${TAG}_pcs.
# Usage (GPU box): TAG=r05d CFG=4 bash tools/gpu/pcsamp.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r05pcs}
RTAMD_LIB=$PWD/raytracing-project_amd/lib/exp/librtamd_dbg.so timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled \
  --pc-sampling-method ${PCS_METHOD:-stochastic} --pc-sampling-unit ${PCS_UNIT:-cycles} --pc-sampling-interval ${PCS_INTERVAL:-1048576} \
  -d gpurun_out/${T}_pcs -o run --output-format csv -- python3 tools/one_frame.py --config ${CFG:-4} --frames ${FRAMES:-6} \
  > gpurun_out/${T}_pcs.log 2>&1
rc=$?
tail -5 gpurun_out/${T}_pcs.log
find gpurun_out/${T}_pcs -type f | head
exit $rc
