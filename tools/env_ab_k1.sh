#!/bin/bash
# configs[1] step time per environment variant, each run twice: tools/env_ab_k1.sh "VAR=val VAR2=val" ...
R=${GRAFT_REPO_ROOT:-/root/repo}
for rep in 1 2; do
for v in "$@"; do
  env $v timeout -k 10 120 python3 $R/bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > /tmp/leg.json 2>/dev/null || exit 1
  python3 -c "
import json,sys; d=json.loads(open('/tmp/leg.json').read().strip().splitlines()[-1])
print(sys.argv[1], round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_isolated'],4))" "$v"
done
done
