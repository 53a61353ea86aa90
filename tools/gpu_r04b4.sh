# round-4 b4: all-pairs shard balance (8 shards), query blocks dealt singly (product) vs in chunks of 4 / 16
mkdir -p gpurun_out
for gen in clustered_traces synth_traces; do
  for v in product chunk4 chunk16; do
    if [ $v = product ]; then unset NMZ_LIB_PATH; else export NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so; fi
    timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/r04b4_bal_${gen}_$v.json 2> gpurun_out/r04b4_bal_${gen}_$v.log || { tail -5 gpurun_out/r04b4_bal_${gen}_$v.log; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/r04b4_bal_${gen}_$v.json'));print('$gen $v', 'unsharded', round(d['unsharded_ms'],2), 'sum', round(d['sum_shard_ms'],2), 'ratio', round(d['sum_shard_ms']/d['unsharded_ms'],3), 'bound', round(d['speedup_bound'],2), 'max/mean', round(d['time_max_over_mean'],3), 'filter', round(sum(r['filter_ms'] for r in d['per_shard']),2), 'dp', round(sum(r['dp_ms'] for r in d['per_shard']),2))"
  done
done
unset NMZ_LIB_PATH
