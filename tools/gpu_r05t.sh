#!/bin/bash
# K1 rank blocks of 128 / 64 / 32 ranks: the K1 and sweep GPU tests, then the headline leg at each width
# (NMZ_WT_BB caps the plan's choice, A/B knob). usage: tools/gpu_r05t.sh <tag> [skip-tests]
tag=${1:-r05t}
O=gpurun_out/$tag
mkdir -p $O
if [ "$2" != "skip-tests" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_sweeps_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/sweeps_tests.log 2>&1
  rc=$?; tail -2 $O/sweeps_tests.log; [ $rc -eq 0 ] || exit $rc
fi
for rep in 1 2; do
for bb in 7 6 5; do
  NMZ_AB=1 NMZ_WT_BB=$bb timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --steps 200 --warmup 20 --full-record $O/bb${bb}_$rep.json > $O/bb${bb}_$rep.out 2> $O/bb${bb}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/bb${bb}_$rep.json'));r=d['roofline']
print('bb $bb rep $rep', '%.4e'%d['value'], round(d['ms_per_step'],4), 'k1', round(r['kernel_ms'],4), 'span', round(r.get('kernel_ms_span',0),4), 'plan', d.get('end_to_end',{}).get('plan_ms'))"
done
done
