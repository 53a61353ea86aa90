#!/bin/bash
# timing ablation: the configs[2] DP without publishing in-band results (NMZ_ABL_PUBLISH build; results wrong)
tag=${1:-r05zj}
O=gpurun_out/$tag
mkdir -p $O
for v in main nopub main nopub; do
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && L=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$L timeout -k 10 300 python bench.py --legs ed_clustered,ed_alphabet --no-cpu-baseline --full-record $O/ed_$v.json > /dev/null 2> $O/ed_$v.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/ed_$v.json'))
for s in d['secondary']: print('$v', s['leg'], round(s['ms_per_step'],3), {k:round(v,3) for k,v in s.get('phases_ms',{}).items()})"
done
