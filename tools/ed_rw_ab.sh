#!/bin/bash
# k_ed_bv block-row size A/B: kernel time per NMZ_ED_RW, then FETCH_SIZE / WRITE_SIZE of the default (one pass each)
R=${GRAFT_REPO_ROOT:-/root/repo}
GEN=${1:-clustered}
bash $R/tools/env_ab_ed.sh $GEN 100000 "NMZ_ED_RW=1" "NMZ_ED_RW=5" "NMZ_ED_RW=10" "NMZ_ED_RW=5" || exit 1
cd /tmp && export TMPDIR=/tmp
for rw in 1 5; do
  for c in FETCH_SIZE WRITE_SIZE; do
    NMZ_ED_RW=$rw timeout -s KILL 200 rocprofv3 --pmc $c --output-format csv -d $R/gpurun_out/edrw_${GEN}_${rw}_$c -o run -- python3 $R/tools/ed_probe.py 100000 2048 32 8 1 $GEN > /dev/null 2>&1 || exit 1
  done
done
echo done
