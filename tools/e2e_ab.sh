# usage: bash tools/e2e_ab.sh <tag> <rounds> <variant>...: configs[1] leg with 17 end-to-end traces, the product
# library vs each namazu_amd/libnmz_gpu_<variant>.so; prints step, plan and end-to-end (one at a time, streamed)
tag=$1; n=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in product "$@"; do
    if [ $v = product ]; then L=""; else L="NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so"; fi
    env $L timeout -k 10 180 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 17 --steps 50 > gpurun_out/${tag}_${v}_$i.json 2>/dev/null || exit $?
  done
done
for f in gpurun_out/${tag}_*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);e=d['end_to_end'];s=d.get('end_to_end_stream') or {}
print('$f', round(d['ms_per_step'],4), 'plan', round(d['plan_ms'],4), 'e2e', round(e['ms_median'],4), '%.3g'%e['value'], 'stream', round(s.get('ms_per_trace',0),4), '%.3g'%s.get('value',0), s.get('agrees_with_one_at_a_time'), 'sides', round(s.get('plan_ms',0),4), round(s.get('sweep_ms',0),4), round(s.get('destroy_ms',0),4), round(s.get('wait_ms',0),4))"; done
