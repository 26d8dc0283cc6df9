# The `ray` CLI on config 4: three fresh timed processes (--stats), then one under
# rocprofv3 with the kernel and HIP API traces (no counters), for the first-frame split.
# Usage (GPU box): TAG=r06c bash tools/gpu/cli_prof.sh
set -o pipefail
export TMPDIR=/tmp
T=${TAG:-r06c}
python3 -c "
import sys; sys.path.insert(0,'raytracing-project_amd/python')
import scenes; t,m=scenes.config_json(4); open('/tmp/c4.json','w').write(t)"
timeout -k 10 120 python3 tools/cli_time.py 4 > gpurun_out/${T}_cli_time.txt 2>&1 || { tail gpurun_out/${T}_cli_time.txt; exit 1; }
cat gpurun_out/${T}_cli_time.txt
RT_CLI_NORMAL_EXIT=1 timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace --stats -d gpurun_out/${T}_prof -o run --output-format csv -- raytracing-project_amd/bin/ray /tmp/c4.json /tmp/o.png --stats --threads 16 > gpurun_out/${T}_prof.log 2>&1 || { tail gpurun_out/${T}_prof.log; exit 1; }
tail -3 gpurun_out/${T}_prof.log
ls -R gpurun_out/${T}_prof | head -20
