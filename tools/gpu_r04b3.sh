# round-4 b3: all-pairs shard balance (8 shards) vs the DP work-item size, both configs[2] generators
mkdir -p gpurun_out
for gen in clustered_traces synth_traces; do
  for it in 4096 2048 1024 512; do
    NMZ_ED_ITEM=$it timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/r04b3_bal_${gen}_$it.json 2> gpurun_out/r04b3_bal_${gen}_$it.log || { tail -5 gpurun_out/r04b3_bal_${gen}_$it.log; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/r04b3_bal_${gen}_$it.json'));print('$gen $it', 'unsharded', round(d['unsharded_ms'],2), 'sum', round(d['sum_shard_ms'],2), 'ratio', round(d['sum_shard_ms']/d['unsharded_ms'],3), 'bound', round(d['speedup_bound'],2), 'max/mean', round(d['time_max_over_mean'],3), 'filter', round(sum(r['filter_ms'] for r in d['per_shard']),2), 'dp', round(sum(r['dp_ms'] for r in d['per_shard']),2))"
  done
done
