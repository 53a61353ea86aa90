#!/bin/bash
# k_trace_sig without the inline rank keys on the common path: visualize GPU tests, then the visualize leg twice
tag=${1:-r05z}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "visual or uniq or trace_sig or PO or por" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  timeout -k 10 200 python bench.py --legs visualize --no-cpu-baseline --full-record $O/vis_$rep.json > /dev/null 2> $O/vis_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/vis_$rep.json'))
for s in d['secondary']: print('$rep', s['leg'], s.get('value'), json.dumps(s.get('roofline',{}))[:300]); print({k:v for k,v in s.items() if 'ms' in k})"
done
