mkdir -p gpurun_out
NMZ_LIB_PATH=$PWD/namazu_amd/libnmz_gpu_wttrace.so timeout -k 10 120 python tools/wt_build_trace.py > gpurun_out/r04t_wt_build_trace.txt 2>&1 || { cat gpurun_out/r04t_wt_build_trace.txt; exit 1; }
cat gpurun_out/r04t_wt_build_trace.txt
bash tools/e2e_ab.sh r04t 2 base
