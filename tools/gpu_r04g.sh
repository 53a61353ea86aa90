mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_ed_gpu.py tests/test_group_gpu.py -x -q --timeout 200 --timeout-method thread -k "entry_limit or plan_from_device or band_routing or group" > gpurun_out/r04g_ed_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04g_ed_tests.log; exit $rc; }
tail -1 gpurun_out/r04g_ed_tests.log
bash tools/k1_check_ab.sh r04g base 3
