# usage: bash tools/lib_ab.sh <tag> <rounds> <variant>...: configs[1] bench leg, the product library vs each
# namazu_amd/libnmz_gpu_<variant>.so, alternating; prints ms/step, K1 alone and K1 span
tag=$1; n=$2; shift 2
mkdir -p gpurun_out
for i in $(seq 1 $n); do
  timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_product_$i.json 2>/dev/null || exit $?
  for v in "$@"; do
    NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_${v}_$i.json 2>/dev/null || exit $?
  done
done
for f in gpurun_out/${tag}_*.json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_isolated'],4), round(d['roofline'].get('kernel_ms') or 0,4))"; done
