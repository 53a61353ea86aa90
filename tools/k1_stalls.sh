#!/bin/bash
# K1 stall counters (one rocprofv3 --pmc pass each) over the headline bench without secondaries.
# usage (GPU box, repo root): tools/k1_stalls.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-k1stalls}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-secondary"
timeout -s KILL 60 rocprofv3 -L > $OUT/avail.txt 2>&1 || true
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA SQ_WAIT_INST_LDS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- $B > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 - "$OUT" <<'PY'
import csv, collections, sys, glob
out = sys.argv[1]
agg = collections.defaultdict(list)
for f in glob.glob(out + "/p*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "replayable_sweep_fast" in r["Kernel_Name"]:
            agg[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(f"{k:28s} {sum(v)/len(v):.4g} per dispatch ({len(v)} rows)")
PY
