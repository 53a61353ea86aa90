#!/bin/bash
# K2 timing per library build: tools/k2_lib_ab.sh lib1.so lib2.so ...  (paths relative to namazu_amd/)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  echo "== $lib"
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 200 python3 $R/tools/k2_probe.py ${K2_S:-1048576} ${K2_REPS:-3} 2>&1 | tail -2 || exit 1
done
