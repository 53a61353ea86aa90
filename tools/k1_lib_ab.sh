#!/bin/bash
# K1 timing per library build: tools/k1_lib_ab.sh lib1.so lib2.so ...  (paths relative to namazu_amd/)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 120 python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > /tmp/k1lib.json 2>/dev/null || exit 1
  python3 -c "import json;d=json.load(open('/tmp/k1lib.json'));print('$lib', 'step_ms', round(d['ms_per_step'],4), 'kernel_ms', round(d['roofline']['kernel_ms'],4), '%.4g' % d['value'])"
done
