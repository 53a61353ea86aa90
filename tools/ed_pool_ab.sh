#!/bin/bash
# ED legs per NMZ_ED_POOL (and other env) variant: tools/ed_pool_ab.sh "VAR=val" ...
R=${GRAFT_REPO_ROOT:-/root/repo}
for v in "$@"; do
  env $v timeout -k 10 300 python3 $R/bench.py --legs ed_clustered,ed_survey --no-cpu-baseline --ed-steps 2 > /tmp/ed.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.load(open('/tmp/ed.json'))
for r in d['secondary']:
    s=r.get('search',{})
    print(sys.argv[1], r['config']['generator'], '%.3e pairs/s'%r['value'], 'kernel_ms', round(r['kernel_ms'],1), 'dp', s.get('dp_pairs'), 'qg', s.get('qgram_settled_pairs'), 'exec cells/s %.3e'%s.get('executed_cells_per_s',0))" "$v"
done
