#!/bin/bash
# rocprofv3 passes over each bench leg separately (kernel names repeat across legs, e.g. k_ed_bv_dp for both
# configs[2] generators); each counter pass is its own run (separate --pmc passes, as MI355X_MICROARCH.md
# prescribes). Also records the machine-code fingerprints of the library that was profiled (isa.json,
# tools/kernel_isa.py) and each leg's bench JSON line (trace.json: the units the kernels processed).
# usage (GPU box, repo root): tools/profile_r03.sh <tag> [legs...]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-prof}; shift || true
LEGS=${*:-replayable random ed_clustered ed_survey ed_alphabet ed_wide visualize}
mkdir -p $R/gpurun_out/$TAG
python3 $R/tools/kernel_isa.py $R/namazu_amd/libnmz_gpu.so $R/gpurun_out/$TAG/isa.json > /dev/null
cd /tmp && export TMPDIR=/tmp
for leg in $LEGS; do
  OUT=$R/gpurun_out/$TAG/$leg
  mkdir -p $OUT
  B="python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --ed-steps 1 --random-steps 1 --e2e-traces 1 --legs $leg"
  echo "== $leg $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $B > $OUT/trace.json 2> $OUT/trace.log
  timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc_valu -o run -- $B > $OUT/pmc_valu.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/pmc_fetch -o run -- $B > $OUT/pmc_fetch.log 2>&1
  timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/pmc_write -o run -- $B > $OUT/pmc_write.log 2>&1
  python3 $R/tools/summarize_profile.py $OUT $OUT/summary.json > $OUT/summary.txt
done
echo done $(date +%T)
