#!/bin/bash
# one bench leg per environment variant: tools/env_ab_bench.sh <leg> "VAR=val" ...  (prints value + kernel_ms)
LEG=$1; shift
R=${GRAFT_REPO_ROOT:-/root/repo}
for v in "$@"; do
  env $v timeout -k 10 300 python3 $R/bench.py --legs $LEG --no-cpu-baseline --random-steps 3 > /tmp/leg.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.load(open('/tmp/leg.json')); s=d['secondary'][0] if 'secondary' in d and d['secondary'] else d
print(sys.argv[1], s.get('value'), s.get('ms_per_step'), s.get('kernel_ms'))" "$v"
done
