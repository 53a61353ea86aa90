#!/bin/bash
# k_trace_sig entity groups from LDS masks (MODE 2) vs ballots (NMZ_SIG_MASKS=0): visualize GPU tests, the
# visualize leg for both, then the visualize leg re-profiled
tag=${1:-r05za}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests -m gpu -k "visual or uniq or trace_sig or PO or por" -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in masks ballots; do
  if [ $v = masks ]; then E=""; else E="NMZ_AB=1 NMZ_SIG_MASKS=0"; fi
  env $E timeout -k 10 200 python bench.py --legs visualize --no-cpu-baseline --full-record $O/${v}_$rep.json > /dev/null 2> $O/${v}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/${v}_$rep.json'))
s=d['secondary'][0]
print('$v $rep', 'po', round(s['po']['sig_kernel_ms'],4), 'exact', round(s['exact']['sig_kernel_ms'],4), 'po value', s['po']['value'])"
done
done
timeout -k 10 600 bash tools/profile_r03.sh ${tag}p visualize > $O/prof.log 2>&1 || exit $?
tail -2 $O/prof.log
