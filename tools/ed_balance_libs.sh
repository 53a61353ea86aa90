#!/bin/bash
# configs[2] 8-shard balance (tools/ed_shard_balance.py) per library variant (namazu_amd/libnmz_gpu_<v>.so; "main" =
# the product library), interleaved. usage: tools/ed_balance_libs.sh <tag> <generator> <reps> <variant>...
tag=$1; gen=$2; reps=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$PWD/namazu_amd/libnmz_gpu_$v.so"; fi
    NMZ_LIB_PATH=$lib timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/${tag}_${gen}_${v}_$i.json 2>> gpurun_out/${tag}.err || exit $?
  done
done
