# usage: bash tools/k1_ab.sh <tag> <variant> [rounds]: configs[1] bench leg, product library (new) vs
# namazu_amd/libnmz_gpu_<variant>.so (old), alternating; prints ms/step and K1 alone
tag=$1; v=$2; n=${3:-2}
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_new$i.json 2>/dev/null || exit $?
  NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_old$i.json 2>/dev/null || exit $?
done
for f in gpurun_out/${tag}_new*.json gpurun_out/${tag}_old*.json; do python3 -c "
import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_isolated'],4), d['roofline'].get('kernel_ms'))"; done
