#!/bin/bash
# headline leg per environment variant (kernel time in the timed region, step time): tools/env_ab_k1.sh "VAR=val" ...
R=${GRAFT_REPO_ROOT:-/root/repo}
for round in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 200 python3 $R/bench.py --legs replayable --no-cpu-baseline --steps 100 --e2e-traces 1 > /tmp/k1.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.load(open('/tmp/k1.json')); r=d['roofline']
print(sys.argv[1], round(d['value']/1e12,3), 'T/s step', round(d['ms_per_step'],4), 'K1', round(r['kernel_ms'],4), 'iso', round(r['kernel_ms_isolated'],4))" "$v"
done
done
