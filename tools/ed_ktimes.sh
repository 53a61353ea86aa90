#!/bin/bash
# ED legs under a rocprofv3 kernel trace: per-dispatch durations of the search kernels. usage: tools/ed_ktimes.sh <tag>
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-edk}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for leg in ed_clustered ed_survey; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$leg -o run -- python3 $R/bench.py --legs $leg --no-cpu-baseline --ed-steps 2 > $OUT/$leg.json 2> $OUT/$leg.err || exit 1
  python3 - "$OUT/$leg" <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/run_kernel_trace.csv", recursive=True)[0]
d = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    n = r["Kernel_Name"]
    if any(k in n for k in ("qg_filter", "qg_scatter", "bv_dp", "k_ed_bv<", "qgram_profile")):
        d[n.split("(")[0]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for n, v in d.items():
    print(sys.argv[1].split("/")[-1], n, ["%.0f us" % x for x in v])
PY
done
