#!/bin/bash
# nmz_replayable_sweep_traces schedules (NMZ_TRACES_MODE 1 = two serial streams, 3 = the Python loop's four-stream
# schedule) against the Python-driven stream, same process each: bench.py's replayable leg. usage: tools/gpu_r05e.sh <tag>
tag=${1:-r05e}; shift; MODES=${*:-1 3}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
  for m in $MODES; do
    NMZ_AB=1 NMZ_TRACES_MODE=$m timeout -k 10 150 python bench.py --legs replayable --no-cpu-baseline --steps 20 --warmup 5 --full-record $O/mode${m}_$rep.json > /dev/null 2> $O/mode${m}_$rep.err || exit $?
  done
done
for f in $O/mode*.json; do python3 -c "
import json;d=json.load(open('$f'));e=d['end_to_end'];n=e['native_batch'];print('$f', 'stream', round(e['ms_per_trace'],4), 'native', round(n['ms_per_trace'],4), n['ms_per_trace_runs'], n['agrees_with_one_at_a_time'])"; done
