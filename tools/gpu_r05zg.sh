#!/bin/bash
# K1 predecessors by a count-guided descent from the root: K1 tests, then the headline leg vs the previous library
tag=${1:-r05zc}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -m gpu  -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in main prev; do
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && L=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$L timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --full-record $O/${v}_$rep.json > /dev/null 2> $O/${v}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/${v}_$rep.json'));r=d['roofline']
print('$v $rep', '%.4e'%d['value'], round(d['ms_per_step'],5), 'k1', round(r['kernel_ms'],4), 'span', round(r.get('kernel_ms_span',0),4))"
done
done
