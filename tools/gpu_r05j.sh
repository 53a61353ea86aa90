#!/bin/bash
# q-gram coarse pre-bound: ED tests, the configs[2] legs (product vs the 6-waves filter build), shard balance.
# usage: tools/gpu_r05j.sh <tag>
tag=${1:-r05j}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ed_gpu.py tests/test_configs_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ed_tests.log 2>&1
rc=$?; tail -2 $O/ed_tests.log; [ $rc -eq 0 ] || exit $rc
for v in main qgw6; do
  lib=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && lib=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --legs ed_survey,ed_clustered --no-cpu-baseline --full-record $O/ed_$v.json > /dev/null 2> $O/ed_$v.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/ed_$v.json'))
for s in d['secondary']: print('$v', s['leg'], round(s['ms_per_step'],3), s.get('phases_ms'), s['roofline'].get('frac'))"
done
bash tools/gpu_r05g.sh $tag auto
