# round-4 checkpoint x: K1 tests (plan kernel: largest segments first, events in LDS), phase trace, end-to-end A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan" > gpurun_out/r04x_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04x_tests.log; exit $rc; }
tail -1 gpurun_out/r04x_tests.log
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04x_trace.txt 2>&1 || { cat gpurun_out/r04x_trace.txt; exit 1; }
cat gpurun_out/r04x_trace.txt
bash tools/e2e_ab.sh r04x 2 NMZ_WT_FUSED=0
