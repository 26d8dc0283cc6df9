# Run each GPU test file in its own pytest process (finds a file whose process aborts at exit).
set -o pipefail
export TMPDIR=/tmp
for t in ${FILES:-tests/test_gpu_parity.py tests/test_gpu_jitter_rows.py tests/test_gpu_dist.py tests/test_gpu_cli.py}; do
  timeout -k 10 300 python -u -m pytest $t -x -q --timeout 120 --timeout-method thread > gpurun_out/bisect.log 2>&1
  rc=$?
  echo "$t rc=$rc $(tail -1 gpurun_out/bisect.log)"
  if [ $rc -ne 0 ]; then tail -20 gpurun_out/bisect.log; exit 1; fi
done
