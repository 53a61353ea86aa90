mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_sweeps_gpu.py tests/test_group_gpu.py tests/test_configs_gpu.py -x -q --timeout 300 --timeout-method thread -k "not config2 and not config4" > gpurun_out/r04k_tests.log 2>&1 || { rc=$?; tail -40 gpurun_out/r04k_tests.log; exit $rc; }
tail -1 gpurun_out/r04k_tests.log
bash tools/k1_ab.sh r04k base 3
