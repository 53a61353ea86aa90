#!/bin/bash
# K1 A/B: sweep parity tests (default variant), then bench per (key, U, EC) variant.
# usage: tools/k1_ab.sh "<key> <U> <EC>" ...   (key = f64 | u64)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
OUT=$R/gpurun_out/k1ab
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest $R/tests/test_sweeps_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
B="python3 $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary"
for cfg in "$@"; do set -- $cfg
  NMZ_REPLAY_KEY=$1 NMZ_REPLAY_U=$2 NMZ_REPLAY_EC=$3 timeout -k 10 120 $B > $OUT/bench_$1_$2_$3.json || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/bench_$1_$2_$3.json')); print('key=$1 U=$2 EC=$3', round(d['ms_per_step'],4), round(d['roofline']['kernel_ms'],4), '%.4g'%d['value'])"; done
