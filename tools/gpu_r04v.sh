# round-4 checkpoint v: replayable (fused plan kernel, separate kernels, order queries) + ED tile tests, the plan
# kernel's phase trace, then the end-to-end A/B: product vs NMZ_WT_FUSED=0 vs the base library
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_sweeps_gpu.py tests/test_ed_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or tile or plan" > gpurun_out/r04v_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04v_tests.log; exit $rc; }
tail -1 gpurun_out/r04v_tests.log
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04v_wt_build_trace.txt 2>&1 || { cat gpurun_out/r04v_wt_build_trace.txt; exit 1; }
cat gpurun_out/r04v_wt_build_trace.txt
bash tools/e2e_ab.sh r04v 2 NMZ_WT_FUSED=0 base
