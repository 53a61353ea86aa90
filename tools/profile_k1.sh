#!/bin/bash
# K1 stall analysis: timing per U variant + SQ wait/active counters (one pass each).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k1
mkdir -p $OUT
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
for u in 2 4 8; do NMZ_REPLAY_U=$u timeout -k 10 120 $B > $OUT/bench_u$u.json || exit 1; done
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS --output-format csv -d $OUT/pmc1 -o run -- $B > $OUT/pmc1.log 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_SALU SQ_LDS_BANK_CONFLICT SQ_WAVES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc2 -o run -- $B > $OUT/pmc2.log 2>&1 || exit 1
echo done
