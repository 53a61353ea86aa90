#!/bin/bash
# K1 library A/B (GPU box): configs[1] step parts and the replayable leg for the product library and variants
# usage: tools/wt_lib_ab.sh <tag> <variant>...   (variant = namazu_amd/libnmz_gpu_<variant>.so)
tag=$1; shift
mkdir -p gpurun_out
for v in main "$@"; do
  lib=namazu_amd/libnmz_gpu.so; [ "$v" != main ] && lib=namazu_amd/libnmz_gpu_$v.so
  for rep in 1 2; do
    NMZ_LIB_PATH=$PWD/$lib timeout -k 10 120 python tools/k1_step_parts.py > gpurun_out/${tag}_${v}_parts$rep.json 2>/dev/null || exit $?
    NMZ_LIB_PATH=$PWD/$lib timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 3 > gpurun_out/${tag}_${v}_bench$rep.json 2>/dev/null || exit $?
  done
done
