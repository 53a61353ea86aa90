#!/bin/bash
# ED timing per env variant (no tests): tools/ed_env_ab.sh "VAR=val" ...
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for cfg in "$@"; do
  echo "== $cfg"
  env $cfg timeout -k 10 250 python3 $R/tools/ed_probe.py ${ED_N:-32768} ${ED_L:-2048} ${ED_W:-32} 8 ${ED_REPS:-3} ${ED_GEN:-} 2>&1 | grep -E "rep [1-9]|kernel avg" | tail -2 || exit 1
done
