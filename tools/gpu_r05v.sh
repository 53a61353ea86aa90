#!/bin/bash
# kernel traces of the headline leg at rank-block widths 5 and 6 (NMZ_WT_BB), to see which step kernels change
tag=${1:-r05v}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$tag
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for bb in 5 6; do
  NMZ_AB=1 NMZ_WT_BB=$bb timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/bb$bb -o run -- python3 $R/bench.py --legs replayable --no-cpu-baseline --steps 100 --warmup 10 --full-record $O/bb$bb.json > $O/bb$bb.out 2> $O/bb$bb.log || exit $?
done
for bb in 5 6; do echo "== bb $bb"; f=$(ls $O/bb$bb/*/run_kernel_stats.csv 2>/dev/null || ls $O/bb$bb/run_kernel_stats.csv); python3 -c "
import csv,sys
for r in sorted(csv.DictReader(open('$f')), key=lambda r:-float(r['TotalDurationNs']))[:12]:
    print('%-50s %6s %9.2f %9.2f'%(r['Name'][:50], r['Calls'], float(r['AverageNs'])/1e3, float(r['TotalDurationNs'])/1e6))"; done
