#!/bin/bash
# configs[1] step helpers: seed-prefix seeds per thread (NMZ_PREFIX_PT) and scatter entries per thread
# (NMZ_SCATTER_PT), A/B knobs; the headline leg, two reps
tag=${1:-r05zk}
O=gpurun_out/$tag
mkdir -p $O
for rep in 1 2; do
for v in 8:16 16:16 4:16 8:8; do
  P=${v%%:*}; S=${v##*:}
  NMZ_AB=1 NMZ_PREFIX_PT=$P NMZ_SCATTER_PT=$S timeout -k 10 200 python bench.py --legs replayable --no-cpu-baseline --full-record $O/p${P}_s${S}_$rep.json > /dev/null 2> $O/p${P}_s${S}_$rep.err || exit $?
  python3 -c "
import json;d=json.load(open('$O/p${P}_s${S}_$rep.json'))
print('ppt $P spt $S rep $rep', '%.4e'%d['value'], round(d['ms_per_step'],5))"
done
done
