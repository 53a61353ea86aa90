#!/bin/bash
# headline step time per pipeline depth: tools/pipeline_ab.sh 2 3 4 ...
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for np in "$@"; do
  NMZ_BENCH_PIPELINE=$np timeout -k 10 120 python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-secondary > /tmp/pl.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/pl.json'));print('pipeline $np', 'step_ms', round(d['ms_per_step'],4), '%.4g' % d['value'])"
done
