# r06i (parity subset + kernel A/B), then the CLI with and without the device warm-up thread.
set -o pipefail
export TMPDIR=/tmp
bash tools/gpu/r06i.sh || exit 1
for w in 1 0 1 0; do
  RAY_WARM_DEVICE=$w timeout -k 10 120 python3 tools/cli_time.py 4 > gpurun_out/r06j_cli_w$w.txt 2>&1 || { tail gpurun_out/r06j_cli_w$w.txt; exit 1; }
  echo "warm_device=$w"; grep render gpurun_out/r06j_cli_w$w.txt | python3 -c "
import sys, json, re
for l in sys.stdin:
    m = re.match(r'render rc 0: ([0-9.]+) ms  (\{.*?\})  (\{.*\})', l.strip())
    if m:
        a = json.loads(m.group(2)); b = json.loads(m.group(3))
        print(' total', m.group(1), 'hip_init', a['ms_hip_init'], 'scene', a['ms_setup_scene'], 'jtable', a['ms_setup_jtable'], 'begin', a['ms_frame_begin'], 'end', a['ms_frame_end'], 'kernel', b['ms_kernel'], 'd2h', b['ms_d2h'], 'png', b['ms_png'], 'render', b['ms_render'])
"
done
