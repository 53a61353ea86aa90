#!/bin/bash
# ED kernel time per environment variant: tools/env_ab_ed.sh <gen> <N> "VAR=val" ...
GEN=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
for v in "$@"; do
  echo "== $v"
  env $v timeout -k 10 300 python3 $R/tools/ed_probe.py $N 2048 32 8 2 $GEN 2>&1 | grep -E "rep 1|kernel avg" || exit 1
done
