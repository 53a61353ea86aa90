#!/bin/bash
# K1 A/B: the row image without pm (timing only, -DWT_ABL_PM: 16 KB less per row) at 1 and 2 workgroups per row
# (NMZ_WT_G; 2 fit one CU only without pm). usage: tools/gpu_r05r.sh <tag>
tag=${1:-r05r}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
for v in ${VARS:-main:1 nopm:1 nopm:2 main:2}; do
  lib=${v%%:*}; G=${v##*:}
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $lib != main ] && L=$PWD/namazu_amd/libnmz_gpu_$lib.so
  NMZ_LIB_PATH=$L NMZ_AB=1 NMZ_WT_G=$G timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --steps 200 --warmup 20 --full-record $O/${lib}_g${G}_$rep.json > $O/${lib}_g${G}_$rep.out 2> $O/${lib}_g${G}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/${lib}_g${G}_$rep.json'));r=d['roofline']
print('$lib G=$G rep $rep', '%.4e'%d['value'], round(d['ms_per_step'],4), 'k1', round(r['kernel_ms'],4), 'span', round(r.get('kernel_ms_span',0),4))"
done
done
