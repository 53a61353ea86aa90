# round-4 b7: ED tests with survivor records for the q-gram scatter, then shard balance (8 shards)
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ed_gpu.py tests/test_group_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04b7_ed_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04b7_ed_tests.log; exit $rc; }
tail -1 gpurun_out/r04b7_ed_tests.log
for gen in clustered_traces synth_traces; do
  timeout -k 10 300 python tools/ed_shard_balance.py $gen 8 > gpurun_out/r04b7_bal_${gen}.json 2> gpurun_out/r04b7_bal_${gen}.log || { tail -5 gpurun_out/r04b7_bal_${gen}.log; exit 1; }
  python3 -c "
import json;d=json.load(open('gpurun_out/r04b7_bal_${gen}.json'));print('$gen', 'unsharded', round(d['unsharded_ms'],2), 'sum', round(d['sum_shard_ms'],2), 'ratio', round(d['sum_shard_ms']/d['unsharded_ms'],3), 'bound', round(d['speedup_bound'],2), 'max/mean', round(d['time_max_over_mean'],3), 'filter', round(sum(r['filter_ms'] for r in d['per_shard']),2), 'dp', round(sum(r['dp_ms'] for r in d['per_shard']),2))"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r04b7_prof -o run -- python3 bench.py --legs ed_survey,ed_clustered --steps 2 --warmup 1 --no-cpu-baseline --ed-steps 1 --e2e-traces 1 > gpurun_out/r04b7_prof.log 2>&1 || exit 1
