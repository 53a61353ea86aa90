#!/bin/bash
# Stall / LDS counters for one kernel of one bench leg (one rocprofv3 --pmc pass per counter set).
# usage (GPU box, repo root): tools/leg_stalls.sh <tag> <leg> <kernel-name-substring>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-stalls}
LEG=${2:-ed_clustered}
KN=${3:-k_ed_bv}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --ed-steps 1 --random-steps 1 --e2e-traces 1 --legs $LEG"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" "$KN" <<'PY'
import csv, collections, sys, glob
out, kn = sys.argv[1], sys.argv[2]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if kn in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):.4g} per dispatch ({len(v)} rows)")
PY
