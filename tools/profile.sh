#!/bin/bash
# rocprofv3 passes over the bench workload; each counter pass is its own run.
# usage (on the GPU box, from the repo root): tools/profile.sh <tag> [extra bench.py args]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}; shift || true
OUT=$R/gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --ed-steps 1 $*"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu -o run -- $B > $OUT/pmc_valu.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1
python3 $R/tools/summarize_profile.py $OUT $OUT/summary.json > $OUT/summary.txt
python3 $R/tools/valu_per_unit.py $OUT/summary.json $TAG > $OUT/valu_per_unit.txt
echo done
