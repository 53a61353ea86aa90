# usage: bash tools/k1_env_ab.sh <tag> <rounds> "<ENV=.. ...>" ["<ENV=..>" ...]: configs[1] bench leg under each
# environment (the first is usually "" = defaults), alternating; prints ms/step, K1 alone and K1 span
tag=$1; n=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  k=0
  for envs in "$@"; do
    k=$((k+1))
    env $envs timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_v${k}_$i.json 2>/dev/null || exit $?
  done
done
k=0
for envs in "$@"; do
  k=$((k+1))
  for f in gpurun_out/${tag}_v${k}_*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('[$envs]', '$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_isolated'],4), round(d['roofline'].get('kernel_ms') or 0,4))"; done
done
