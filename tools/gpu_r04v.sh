# round-4 checkpoint v: replayable + ED tile tests, then the end-to-end A/B (streamed side timings)
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sweeps_gpu.py tests/test_ed_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or tile or plan" > gpurun_out/r04v_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04v_tests.log; exit $rc; }
tail -1 gpurun_out/r04v_tests.log
bash tools/e2e_ab.sh r04v 2 base
