#!/bin/bash
# the driver's own bench command (python bench.py, defaults) twice on HEAD, then the headline leg with 32-rank blocks
tag=${1:-r05y}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python bench.py --full-record $O/full_$rep.json > $O/bench_$rep.out 2> $O/bench_$rep.err || exit $?
  python3 -c "
import json;d=json.loads(open('$O/bench_$rep.out').read().strip().splitlines()[-1]);r=d['roofline']
print('default rep $rep', '%.4e'%d['value'], d['ms_per_step'], 'k1', r['kernel_ms'], 'span', r.get('kernel_ms_span'), 'frac', r.get('frac'))"
done
NMZ_AB=1 NMZ_WT_BB=5 timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --full-record $O/bb5.json > $O/bb5.out 2> $O/bb5.err || exit $?
python3 -c "
import json;d=json.load(open('$O/bb5.json'));r=d['roofline']
print('bb5 leg', '%.4e'%d['value'], d['ms_per_step'], 'k1', r['kernel_ms'])"
