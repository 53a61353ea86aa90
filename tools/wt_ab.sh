#!/bin/bash
# K1 wavelet-tree launch shape A/B (GPU box, repo root): workgroups per row x threads per workgroup, replayable leg
mkdir -p gpurun_out
tag=${1:-wt_ab}
for cfg in "1 1024" "2 1024" "2 512" "4 512" "4 256" "8 256" "8 512" "4 1024"; do
  set -- $cfg
  NMZ_WT_G=$1 NMZ_WT_THREADS=$2 timeout -k 10 120 python bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 \
    > gpurun_out/${tag}_g$1_t$2.json 2>/dev/null || exit $?
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --legs replayable --no-cpu-baseline --e2e-traces 1 > $GRAFT_REPO_ROOT/gpurun_out/${tag}_prof.json 2>&1
