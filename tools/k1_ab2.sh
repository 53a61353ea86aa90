#!/bin/bash
# K1 A/B per library build, pipelined (3 streams) and unpipelined: tools/k1_ab2.sh lib1.so lib2.so ...
# (paths relative to namazu_amd/); prints step time, K1 span per launch and K1 alone
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  for np in ${PIPES:-3 1}; do
    NMZ_BENCH_PIPELINE=$np NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 120 python3 $R/bench.py --steps 100 --warmup 5 --no-cpu-baseline --no-secondary > /tmp/k1lib.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('/tmp/k1lib.json'));r=d['roofline'];print('$lib', 'pipe', $np, 'step_ms', round(d['ms_per_step'],4), 'span_ms', round(r['kernel_ms'],4), 'isolated_ms', round(r['kernel_ms_isolated'],4), '%.4g' % d['value'])"
  done
done
