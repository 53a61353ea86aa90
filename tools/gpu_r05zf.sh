#!/bin/bash
# configs[1] pipeline depth (NMZ_BENCH_PIPELINE 2 / 3 (default) / 4): the headline leg, two reps
tag=${1:-r05zf}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
for p in 3 4 2; do
  NMZ_BENCH_PIPELINE=$p timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --full-record $O/p${p}_$rep.json > /dev/null 2> $O/p${p}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/p${p}_$rep.json'));r=d['roofline']
print('pipe $p rep $rep', '%.4e'%d['value'], round(d['ms_per_step'],5), 'k1', round(r['kernel_ms'],4), 'span', round(r.get('kernel_ms_span',0),4))"
done
done
