# usage: bash tools/gpu_oq.sh <tag>: K1 parity tests, then the configs[1] bench leg with the order-query
# statistics (default) and with the per-decision sweep (NMZ_REPLAY_OQ=0)
tag=$1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py tests/test_configs_gpu.py -k "replayable or config1 or topk or random" \
  -x -v --timeout 120 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${tag}_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 200 python bench.py --legs replayable > gpurun_out/${tag}_bench_oq.json 2> gpurun_out/${tag}_bench_oq.err || exit $?
NMZ_REPLAY_OQ=0 timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline > gpurun_out/${tag}_bench_dec.json 2> gpurun_out/${tag}_bench_dec.err
