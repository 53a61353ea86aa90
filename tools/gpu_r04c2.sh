# round-4 c2: K1 tests with the split plan launch (small segments on a second stream), phase trace, e2e A/B
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan or topk" > gpurun_out/r04c2_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04c2_tests.log; exit $rc; }
tail -1 gpurun_out/r04c2_tests.log
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04c2_trace.txt 2>&1 || { cat gpurun_out/r04c2_trace.txt; exit 1; }
cat gpurun_out/r04c2_trace.txt
bash tools/e2e_ab.sh r04c2 2 NMZ_WT_SMALL=0
