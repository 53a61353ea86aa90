#!/bin/bash
# A/B of library variants on the ED all-pairs kernel: tools/ab_ed.sh <gen> <N> lib1.so lib2.so ... (relative to namazu_amd/)
GEN=$1; N=$2; shift 2
R=${GRAFT_REPO_ROOT:-/root/repo}
for round in 1 2; do
for lib in "$@"; do
  echo "== $lib round $round"
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 300 python3 $R/tools/ed_probe.py $N 2048 32 8 3 $GEN 2>&1 | grep -E "rep 2|kernel avg" || exit 1
done
done
