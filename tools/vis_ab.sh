#!/bin/bash
# visualize leg A/B per library build: tools/vis_ab.sh lib1.so lib2.so ... (paths relative to namazu_amd/)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 200 python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --legs replayable,visualize > /tmp/vis.json 2>/dev/null || exit 1
  python3 -c "
import json;b=json.load(open('/tmp/vis.json'))
v=[s for s in b['secondary'] if 'visualize' in s.get('config',{}).get('workload','')][0]
print('$lib', 'po sig_ms', round(v['po']['sig_kernel_ms'],4), 'GB/s', round(v['po']['roofline']['achieved']), 'curve_ms', round(v['po']['ms'],4), '| exact sig_ms', round(v['exact']['sig_kernel_ms'],4), 'GB/s', round(v['exact']['roofline']['achieved']), 'unique', v['po']['unique'], v['exact']['unique'])"
done
