#!/bin/bash
# ED A/B: bit-parallel parity tests, then ed_probe per env variant: tools/ed_ab.sh "VAR=val" ...
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
timeout -k 10 300 python3 -u -m pytest $R/tests/test_ed_gpu.py -x -q --timeout 120 --timeout-method thread > $R/gpurun_out/ed_ab_tests.log 2>&1 || { tail -30 $R/gpurun_out/ed_ab_tests.log; exit 1; }
tail -1 $R/gpurun_out/ed_ab_tests.log
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 200 python3 $R/tools/ed_probe.py ${ED_N:-32768} 2048 32 8 3 2>&1 | grep -E "rep 2|kernel avg" || exit 1
done
