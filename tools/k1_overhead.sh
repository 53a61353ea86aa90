#!/bin/bash
# per-kernel stats of the replayable step under env variants: tools/k1_overhead.sh "VAR=val VAR2=val" ...
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/k1oh
mkdir -p $OUT
i=0
for cfg in "$@"; do
  i=$((i+1))
  echo "== $cfg"
  env $cfg timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/v$i -o run -- python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary > $OUT/v$i.json 2> $OUT/v$i.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/v$i.json'));print('step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4))"
  python3 $R/tools/kstats.py $OUT/v$i/run_kernel_stats.csv
done
