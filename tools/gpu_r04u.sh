mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_sweeps_gpu.py -x -q --timeout 200 --timeout-method thread -k "k1 or wt or replayable" > gpurun_out/r04u_k1_tests.log 2>&1 || { rc=$?; tail -30 gpurun_out/r04u_k1_tests.log; exit $rc; }
tail -1 gpurun_out/r04u_k1_tests.log
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04u_wt_build_trace.txt 2>&1 || { cat gpurun_out/r04u_wt_build_trace.txt; exit 1; }
cat gpurun_out/r04u_wt_build_trace.txt
bash tools/e2e_ab.sh r04u 2 base
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for v in product base; do
  if [ $v = product ]; then unset NMZ_LIB_PATH; else export NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_base.so; fi
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r04u_tile_$v -o run -- python3 tools/tile_ab.py > gpurun_out/r04u_tile_$v.log 2>&1 || { tail -20 gpurun_out/r04u_tile_$v.log; exit 1; }
  cat gpurun_out/r04u_tile_$v.log | grep band
done
unset NMZ_LIB_PATH
