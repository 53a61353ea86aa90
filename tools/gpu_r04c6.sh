# round-4 c6: K1 tests incl. the native multi-trace sweep, then the end-to-end runs
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan or topk or seed" > gpurun_out/r04c6_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04c6_tests.log; exit $rc; }
tail -1 gpurun_out/r04c6_tests.log
bash tools/e2e_ab.sh r04c6 2
