#!/bin/bash
# q-gram filter: survivor records counted in 64 striped counters instead of one: ED tests, then the configs[2] legs
# against the previous library, then the 8-shard balance
tag=${1:-r05zh}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ed_gpu.py tests/test_configs_gpu.py tests/test_group_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ed_tests.log 2>&1
rc=$?; tail -2 $O/ed_tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
for v in main prev; do
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && L=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$L timeout -k 10 300 python bench.py --legs ed_survey,ed_clustered,ed_alphabet --no-cpu-baseline --full-record $O/ed_${v}_$rep.json > /dev/null 2> $O/ed_${v}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/ed_${v}_$rep.json'))
for s in d['secondary']: print('$v $rep', s['leg'], round(s['ms_per_step'],3), {k:round(v,3) for k,v in s.get('phases_ms',{}).items()})"
done
done
bash tools/gpu_r05g.sh $tag auto
