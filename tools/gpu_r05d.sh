#!/bin/bash
# configs[2] shard anatomy (GPU box): tools/ed_shard_balance.py on both generators with a kernel trace, and one
# FETCH_SIZE pass each (DP traffic per launch: unsharded vs the 8 shards). usage: tools/gpu_r05d.sh <tag>
tag=${1:-r05d}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for g in clustered_traces synth_traces; do
  mkdir -p $O/$g
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$g/trace -o run -- python3 $R/tools/ed_shard_balance.py $g 8 > $O/$g/bal.json 2> $O/$g/bal.log || exit $?
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/$g/fetch -o run -- python3 $R/tools/ed_shard_balance.py $g 8 > $O/$g/bal_fetch.json 2> $O/$g/fetch.log || exit $?
done
exit 0
