#!/bin/bash
# configs[2] shard balance A/B (GPU box): dealing (snake / hash) x DP item size, 8 shards, both generators
tag=${1:-edbal}
mkdir -p gpurun_out
for deal in snake hash; do
  for item in 4096 1024; do
    for gen in clustered_traces synth_traces; do
      NMZ_ED_DEAL=$deal NMZ_ED_ITEM=$item timeout -k 10 200 python tools/ed_shard_balance.py $gen 8 \
        > gpurun_out/${tag}_${deal}_${item}_${gen}.json 2>/dev/null || exit $?
    done
  done
done
