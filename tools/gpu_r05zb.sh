#!/bin/bash
# k_trace_sig PO: steps loaded together per wave (NMZ_SIG_U 2 / 4 (product) / 8), the visualize leg
tag=${1:-r05zb}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
for v in main u8 u2; do
  L=$PWD/namazu_amd/libnmz_gpu.so; [ $v != main ] && L=$PWD/namazu_amd/libnmz_gpu_$v.so
  NMZ_LIB_PATH=$L timeout -k 10 200 python bench.py --legs visualize --no-cpu-baseline --full-record $O/${v}_$rep.json > /dev/null 2> $O/${v}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/${v}_$rep.json'))
s=d['secondary'][0]
print('$v $rep', 'po', round(s['po']['sig_kernel_ms'],4), 'exact', round(s['exact']['sig_kernel_ms'],4))"
done
done
