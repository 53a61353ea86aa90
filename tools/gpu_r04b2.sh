# round-4 checkpoint b2: ED tests with the superblock tile order, then shard balance (8 shards) for both configs[2]
# generators, product vs base library
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ed_gpu.py tests/test_group_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b2_ed_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04b2_ed_tests.log; exit $rc; }
tail -1 gpurun_out/r04b2_ed_tests.log
for gen in clustered_traces survey_traces; do
  for v in product base; do
    if [ $v = product ]; then unset NMZ_LIB_PATH; else export NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_base.so; fi
    timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/r04b2_bal_${gen}_$v.json 2> gpurun_out/r04b2_bal_${gen}_$v.log || { tail -5 gpurun_out/r04b2_bal_${gen}_$v.log; exit 1; }
    python3 -c "
import json;d=json.load(open('gpurun_out/r04b2_bal_${gen}_$v.json'));print('$gen $v', 'unsharded', round(d['unsharded_ms'],2), 'sum', round(d['sum_shard_ms'],2), 'ratio', round(d['sum_shard_ms']/d['unsharded_ms'],3), 'bound', round(d['speedup_bound'],2), 'filter', [round(r['filter_ms'],2) for r in d['per_shard']], 'dp', [round(r['dp_ms'],2) for r in d['per_shard']])"
  done
done
unset NMZ_LIB_PATH
