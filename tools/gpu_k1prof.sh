# usage: bash tools/gpu_k1prof.sh <tag>: kernel trace + stall/LDS counters of the configs[1] leg
tag=$1
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/$tag/trace -o run -- \
  python3 $R/bench.py --steps 20 --warmup 2 --no-cpu-baseline --e2e-traces 1 --legs replayable > $R/gpurun_out/$tag/trace.log 2>&1 || exit $?
cd $R && bash tools/leg_stalls.sh $tag/stalls replayable k_replayable_sweep_oq > gpurun_out/$tag/stalls.txt 2>&1
