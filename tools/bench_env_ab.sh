#!/bin/bash
# headline bench per env variant (no CPU baseline / secondary legs): tools/bench_env_ab.sh "VAR=val" ...
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
i=0
for cfg in "$@"; do
  i=$((i+1))
  env $cfg timeout -k 10 120 python3 $R/bench.py --steps ${STEPS:-50} --warmup 3 --no-cpu-baseline --no-secondary > $R/gpurun_out/benv$i.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('$R/gpurun_out/benv$i.json'));print('$cfg', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])"
done
