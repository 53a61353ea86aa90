#!/bin/bash
# configs[2] legs A/B per library build: tools/ed_filter_ab.sh lib1.so lib2.so ... (paths relative to namazu_amd/)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 300 python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --legs replayable,ed_clustered,ed_survey > /tmp/edab.json 2>/dev/null || exit 1
  python3 -c "
import json;b=json.load(open('/tmp/edab.json'))
for s in b['secondary']:
  if 'configs[2]' in s.get('config',{}).get('workload',''):
    print('$lib', s['config']['generator'][:10], 'ms', round(s['ms_per_step'],2), 'phases', {k: round(v,2) for k,v in s['phases_ms'].items()}, 'qgram', s['search']['qgram_settled_pairs'], 'inband', s['search']['in_band_pairs'], 'agree', s['single_query']['agrees_with_allpairs'])"
done
