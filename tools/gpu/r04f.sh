# Round-4: light-centred shadow culls: full GPU suite, bench, kernel trace + instruction mix (config 4).
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r04f}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.log 2>&1 || { echo "tests failed"; grep -E "FAIL|Error|assert" gpurun_out/${T}_gpu_tests.log | head -30; tail -30 gpurun_out/${T}_gpu_tests.log; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.log
timeout -k 10 300 python bench.py --steps 200 --no-cpu --no-pmc --no-cli > gpurun_out/${T}_bench.json 2> gpurun_out/${T}_bench.err || { echo bench failed; tail gpurun_out/${T}_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/${T}_bench.json')); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel_ms'], r['frac'], r['executed_frac'], r['occupancy'])"
for c in 5 6 3; do
  timeout -k 10 200 python3 tools/one_frame.py --config $c --frames 1 > /dev/null 2>&1
done
timeout -k 10 400 bash tools/gpu/pmc_detail.sh 4 > gpurun_out/${T}_pmc_detail_cfg4.txt 2>&1 || { echo "pmc failed"; tail gpurun_out/${T}_pmc_detail_cfg4.txt; exit 1; }
grep -E "k_std|SQ_INSTS_VALU  |SQ_INSTS_VALU |SQ_INSTS_SALU|SQ_WAVES" gpurun_out/${T}_pmc_detail_cfg4.txt | head
