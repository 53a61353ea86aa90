mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "k1 or wt or replayable" > gpurun_out/r04o_k1_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04o_k1_tests.log; exit $rc; }
tail -1 gpurun_out/r04o_k1_tests.log
bash tools/k1_env_ab.sh r04o 3 "" "NMZ_WT_NS=1"
