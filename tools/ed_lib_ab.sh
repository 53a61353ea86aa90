#!/bin/bash
# ED timing per library build: tools/ed_lib_ab.sh lib1.so lib2.so ...  (paths relative to namazu_amd/)
cd /tmp && export TMPDIR=/tmp
R=${GRAFT_REPO_ROOT:-/root/repo}
for lib in "$@"; do
  echo "== $lib"
  NMZ_LIB_PATH=$R/namazu_amd/$lib timeout -k 10 200 python3 $R/tools/ed_probe.py ${ED_N:-32768} ${ED_L:-2048} ${ED_W:-32} 8 3 ${ED_GEN:-} 2>&1 | grep -E "rep 2|kernel avg" || exit 1
done
