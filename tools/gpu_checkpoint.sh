# usage: bash tools/gpu_checkpoint.sh <tag>: the whole -m gpu suite, smoke(), then the default bench (all legs)
tag=$1
mkdir -p gpurun_out
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_gpu_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/${tag}_gpu_tests.log; exit $rc; }
tail -1 gpurun_out/${tag}_gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${tag}_smoke.log 2>&1 || { rc=$?; tail -20 gpurun_out/${tag}_smoke.log; exit $rc; }
tail -2 gpurun_out/${tag}_smoke.log
timeout -k 10 900 python bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.log || { rc=$?; tail -20 gpurun_out/${tag}_bench.log; exit $rc; }
python3 -c "
import json;d=json.loads(open('gpurun_out/${tag}_bench.json').read().strip().splitlines()[-1]);e=d['end_to_end'];print(d['value'], d['ms_per_step'], e['value'], e.get('ms_per_trace'), e.get('one_at_a_time', {}).get('value'), d['plan_ms'])"
