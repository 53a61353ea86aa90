#!/bin/bash
# A/B of library variants (namazu_amd/libnmz_gpu_<name>.so, built with make VARIANT=name EXTRA=...) on one bench leg:
# usage: tools/lib_variants_ab.sh <tag> <legs> <reps> <variant>... ("main" = the product library). Runs the variants
# interleaved (reps rounds), each under its own time limit; the full records go to gpurun_out/<tag>_<variant>_<i>.json.
tag=$1; legs=$2; reps=$3; shift 3
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for v in "$@"; do
    if [ "$v" = main ]; then lib=""; else lib="$PWD/namazu_amd/libnmz_gpu_$v.so"; fi
    NMZ_LIB_PATH=$lib timeout -k 10 300 python bench.py --legs "$legs" --no-cpu-baseline \
      --full-record gpurun_out/${tag}_${v}_$i.json > /dev/null 2>> gpurun_out/${tag}.err || exit $?
  done
done
