#!/bin/bash
# K1 iteration: sweep parity tests, then bench per U variant (no CPU baseline / secondary).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/k1try
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest $R/tests/test_sweeps_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for u in ${UVARS:-2 4}; do
  NMZ_REPLAY_U=$u timeout -k 10 120 python $R/bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-secondary > $OUT/bench_u$u.json || exit 1
  python -c "import json;d=json.load(open('$OUT/bench_u$u.json'));print('U=$u', d['ms_per_step'], d['roofline']['kernel_ms'], '%.3e'%d['value'])"
done
