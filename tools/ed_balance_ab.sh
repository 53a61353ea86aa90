#!/bin/bash
# configs[2] 8-shard balance (tools/ed_shard_balance.py) for both generators, with an optional A/B environment for
# the second run of each pair. usage: tools/ed_balance_ab.sh <tag> <reps> ["ENV=value ..."]
tag=$1; reps=$2; abenv=$3
mkdir -p gpurun_out
for i in $(seq 1 $reps); do
  for gen in synth_traces clustered_traces; do
    timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/${tag}_${gen}_main_$i.json 2>> gpurun_out/${tag}.err || exit $?
    if [ -n "$abenv" ]; then
      env NMZ_AB=1 $abenv timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/${tag}_${gen}_ab_$i.json 2>> gpurun_out/${tag}.err || exit $?
    fi
  done
done
