#!/bin/bash
# K1 anatomy on the GPU box: the per-wave timeline of one launch (-DWT_TRACE build) and the serial K1 time of the
# product library against ablation builds (WT_ABL_LIFT / COUNT / PRED skip one part; results wrong, timing only).
# usage: tools/gpu_r05b.sh <tag> [variants...]
tag=${1:-r05b}; shift
O=gpurun_out/$tag
mkdir -p $O
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/k1_trace.py --wt > $O/trace.txt 2>&1 || exit $?
for v in main "$@"; do
  lib=$PWD/namazu_amd/libnmz_gpu.so; [ "$v" != main ] && lib=$PWD/namazu_amd/libnmz_gpu_$v.so
  for rep in 1 2; do
    NMZ_LIB_PATH=$lib timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 2 --steps 20 --warmup 5 --full-record "" > $O/${v}_$rep.json 2>/dev/null || exit $?
  done
done
for f in $O/*_[12].json; do python3 -c "
import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);r=d['roofline'];print('$f', round(d['ms_per_step'],4), round(r['kernel_ms'],4), round(r['kernel_ms_serial_span'],4))"; done
