#!/bin/bash
# K1: segments of <= 32 events as per-event decisions (NMZ_WT_BRUTE=32 build) vs <= 8 (product): K1 tests on the
# variant, then the headline leg for both
tag=${1:-r05ze}
O=gpurun_out/$tag
mkdir -p $O
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_br32.so timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests_br32.log 2>&1
rc=$?; tail -2 $O/tests_br32.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in main br32; do
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && L=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$L timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --full-record $O/${v}_$rep.json > /dev/null 2> $O/${v}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/${v}_$rep.json'));r=d['roofline']
print('$v $rep', '%.4e'%d['value'], round(d['ms_per_step'],5), 'k1', round(r['kernel_ms'],4), 'span', round(r.get('kernel_ms_span',0),4))"
done
done
