set -o pipefail
export TMPDIR=/tmp
timeout -k 10 300 python tools/opcount_parity.py > gpurun_out/opc.log 2>&1 || { echo opc failed; tail -20 gpurun_out/opc.log; exit 1; }
cat gpurun_out/opc.log
