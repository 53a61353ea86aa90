#!/bin/bash
# two-phase offsets in two kernels: ED tests, the configs[2] legs, 8-shard balance, then the ED legs re-profiled
# (their kernels changed). usage: tools/gpu_r05q.sh <tag>
tag=${1:-r05q}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_ed_gpu.py tests/test_configs_gpu.py tests/test_group_gpu.py tests/test_dist_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/ed_tests.log 2>&1
rc=$?; tail -2 $O/ed_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --legs ed_survey,ed_clustered,ed_alphabet --no-cpu-baseline --full-record $O/ed_main.json > /dev/null 2> $O/ed_main.err || exit $?
python3 -c "
import json;d=json.load(open('$O/ed_main.json'))
for s in d['secondary']: print(s['leg'], round(s['ms_per_step'],3), {k:round(v,3) for k,v in s.get('phases_ms',{}).items()})"
bash tools/gpu_r05g.sh $tag auto || exit $?
timeout -k 10 900 bash tools/profile_r03.sh ${tag}p ed_clustered ed_survey ed_alphabet > $O/prof.log 2>&1 || exit $?
tail -3 $O/prof.log
