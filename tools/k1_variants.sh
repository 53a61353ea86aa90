#!/bin/bash
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/k1v
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest $R/tests/test_sweeps_gpu.py -x -q --timeout 300 --timeout-method thread -k replayable > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="python3 $R/bench.py --steps 10 --warmup 2 --no-cpu-baseline --no-secondary"
for cfg in "2 1024" "2 512" "2 2048" "4 1024" "4 512" "2 4096"; do set -- $cfg
  NMZ_REPLAY_U=$1 NMZ_REPLAY_EC=$2 timeout -k 10 120 $B > $OUT/bench_$1_$2.json || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/bench_$1_$2.json')); print('U=$1 EC=$2', round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), '%.3g'%d['value'])"; done
