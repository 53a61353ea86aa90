# round-4 checkpoint w: K1 tests (fused plan kernel with word-wide hint loads), the plan kernel's phase trace with
# and without the per-class rS atomic, then the end-to-end A/B: product vs NMZ_WT_FUSED=0
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "replayable or wt or k1 or plan" > gpurun_out/r04w_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04w_tests.log; exit $rc; }
tail -1 gpurun_out/r04w_tests.log
for v in wttrace wtnoat; do
  NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_$v.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04w_trace_$v.txt 2>&1 || { cat gpurun_out/r04w_trace_$v.txt; exit 1; }
  echo $v; cat gpurun_out/r04w_trace_$v.txt
done
bash tools/e2e_ab.sh r04w 2 NMZ_WT_FUSED=0
