set -o pipefail
python3 -c "
import sys; sys.path.insert(0,'raytracing-project_amd/python')
import scenes; t,m=scenes.config_json(4); open('/tmp/c4.json','w').write(t)"
for i in 1 2; do timeout -k 10 60 raytracing-project_amd/bin/ray /tmp/c4.json /tmp/o.png --stats --threads 16 | tail -2; done
