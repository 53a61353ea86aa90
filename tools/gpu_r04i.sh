mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ed_gpu.py tests/test_group_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04i_ed_tests.log 2>&1 || { rc=$?; tail -40 gpurun_out/r04i_ed_tests.log; exit $rc; }
tail -1 gpurun_out/r04i_ed_tests.log
bash tools/k1_ab.sh r04i base 3
