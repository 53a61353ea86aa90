#!/bin/bash
# kernel timeline of the configs[1] step with the top-k (rocprofv3 kernel trace over tools/k1_step_parts.py)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-k1tk}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- python3 $R/tools/k1_step_parts.py > $OUT/parts.json 2> $OUT/log.txt
