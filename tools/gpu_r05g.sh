#!/bin/bash
# configs[2] shard balance under DP work-item sizes (NMZ_ED_ITEM, A/B knob): 4096 (product) vs smaller items.
# usage: tools/gpu_r05g.sh <tag> <items...>   (auto: the product's choice, no NMZ_ED_ITEM)
tag=${1:-r05g}; shift
O=gpurun_out/$tag
mkdir -p $O
for it in "$@"; do
  for g in clustered_traces synth_traces; do
    if [ "$it" = auto ]; then
      timeout -k 10 200 python tools/ed_shard_balance.py $g 8 > $O/${g}_$it.json 2> $O/${g}_$it.err || exit $?
    else
      NMZ_AB=1 NMZ_ED_ITEM=$it timeout -k 10 200 python tools/ed_shard_balance.py $g 8 > $O/${g}_$it.json 2> $O/${g}_$it.err || exit $?
    fi
  done
done
for f in $O/*_traces_*.json; do python3 -c "
import json;d=json.load(open('$f'));print('$f', round(d['unsharded_ms'],3), round(d['sum_shard_ms'],3), round(d['max_shard_ms'],3), round(d['speedup_bound'],3), 'dp', [round(r['dp_ms'],3) for r in d['per_shard']])"; done
