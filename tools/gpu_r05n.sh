#!/bin/bash
# sparse-item DP path (one query per lane): ED tests, the configs[2] legs product vs nomono, shard balance.
# usage: tools/gpu_r05n.sh <tag>
tag=${1:-r05n}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ed_gpu.py tests/test_configs_gpu.py tests/test_group_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ed_tests.log 2>&1
rc=$?; tail -2 $O/ed_tests.log; [ $rc -eq 0 ] || exit $rc
for v in main nomono; do
  lib=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && lib=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --legs ed_survey,ed_clustered,ed_alphabet --no-cpu-baseline --full-record $O/ed_$v.json > /dev/null 2> $O/ed_$v.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/ed_$v.json'))
for s in d['secondary']: print('$v', s['leg'], round(s['ms_per_step'],3), {k:round(v,3) for k,v in s.get('phases_ms',{}).items()})"
done
bash tools/gpu_r05g.sh $tag auto
