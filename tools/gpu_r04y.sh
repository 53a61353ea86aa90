# round-4 checkpoint y: K1 tests incl. asynchronous plan creation, phase trace, end-to-end A/B (streamed: async)
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan" > gpurun_out/r04y_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04y_tests.log; exit $rc; }
tail -1 gpurun_out/r04y_tests.log
bash tools/e2e_ab.sh r04y 2 NMZ_WT_FUSED=0
