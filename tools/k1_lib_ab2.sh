# usage: bash tools/k1_lib_ab2.sh <tag> <variant>: configs[1] bench leg, product library vs libnmz_gpu_<variant>.so, alternating
tag=$1; v=$2
mkdir -p gpurun_out
for i in 1 2; do
  timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_base$i.json 2>/dev/null || exit $?
  NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > gpurun_out/${tag}_$v$i.json 2>/dev/null || exit $?
done
for f in gpurun_out/${tag}_*.json; do python3 -c "
import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms_isolated'],4))"; done
