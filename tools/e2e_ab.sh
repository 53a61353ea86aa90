# usage: bash tools/e2e_ab.sh <tag> <rounds> <variant>...: configs[1] leg with the default stream of end-to-end traces (64), the product
# library vs each namazu_amd/libnmz_gpu_<variant>.so (or, for a variant VAR=value, the product library with that
# environment setting); prints step, plan and end-to-end (one at a time, streamed)
tag=$1; n=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  for v in product "$@"; do
    if [ $v = product ]; then L=""; elif [[ $v == *=* ]]; then L="$v"; else L="NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so"; fi
    name=${v//=/_}
    env $L timeout -k 10 180 python bench.py --legs replayable --no-cpu-baseline --steps 50 > gpurun_out/${tag}_${name}_$i.json 2>/dev/null || exit $?
  done
done
for f in gpurun_out/${tag}_*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);e=d['end_to_end'];o=e.get('one_at_a_time', e)
print('$f', round(d['ms_per_step'],4), 'plan', round(d['plan_ms'],4), 'one', round(o['ms_median'],4), '%.3g'%o['value'], 'stream', round(e.get('ms_per_trace',0),4), '%.3g'%e['value'], e.get('agrees_with_one_at_a_time'), 'native', round((e.get('native_batch') or {}).get('ms_per_trace',0),4))"; done
