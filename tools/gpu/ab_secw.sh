# A/B of the recursion kernel: head vs cur (and lib/exp/librtamd_<name>.so for each name given) on config 6
# and the no-bounce base (tools/secw_base.py), recursion tests first.
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_recursion.py tests/test_gpu_parity.py tests/test_gpu_deep.py -m gpu -x -q --timeout 300 --timeout-method thread 2>&1 | tail -2 || exit 1
for v in head cur "$@"; do
  case $v in
    cur) L=$PWD/raytracing-project_amd/lib/librtamd.so ;;
    head) L=$PWD/raytracing-project_amd/lib/librtamd_head.so ;;
    *) L=$PWD/raytracing-project_amd/lib/exp/librtamd_$v.so ;;
  esac
  echo "== $v"
  RTAMD_LIB=$L timeout -k 10 300 python tools/secw_base.py 2>&1 | grep -v amdgpu.ids || exit 1
  RTAMD_LIB=$L timeout -k 10 200 python bench.py --config 6 --no-cpu --no-pmc --no-cli --fp32-steps 0 --steps 50 --warmup 3 | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('cfg 6 frame_ms', d['ms_per_step'], 'kernel_ms', d['roofline']['kernel_ms'])" || exit 1
done
