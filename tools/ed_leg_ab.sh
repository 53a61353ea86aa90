#!/bin/bash
# bench.py ED legs per library variant (namazu_amd/libnmz_gpu_<v>.so; "main" = the product library), interleaved.
# usage: tools/ed_leg_ab.sh <tag> <reps> <legs (comma list)> <variant>...
tag=$1; reps=$2; legs=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$PWD/namazu_amd/libnmz_gpu_$v.so"; fi
    for leg in ${legs//,/ }; do
      NMZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --ed-steps 2 --legs $leg > gpurun_out/${tag}_${leg}_${v}_$i.json 2>> gpurun_out/${tag}.err || exit $?
    done
  done
done
