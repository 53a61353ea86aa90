#!/bin/bash
# visualize tests + the visualize leg (k_trace_sig), then the configs[2] item-size A/B. usage: tools/gpu_r05i.sh <tag>
tag=${1:-r05i}
O=gpurun_out/$tag
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_visualize.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/vis_tests.log 2>&1
rc=$?; tail -2 $O/vis_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python bench.py --legs visualize --no-cpu-baseline --full-record $O/vis.json > /dev/null 2> $O/vis.err || exit $?
python3 -c "
import json;d=json.load(open('$O/vis.json'))['secondary'][0]
print('po', round(d['po']['sig_kernel_ms'],4), round(d['po']['roofline']['frac'],3), 'exact', round(d['exact']['sig_kernel_ms'],4), round(d['exact']['roofline']['frac'],3))"
bash tools/gpu_r05g.sh $tag auto 512
