#!/usr/bin/env python3
"""K1 launch timeline from a rocprofv3 kernel_trace.csv (usage: k1_timeline.py <kernel_trace.csv> [kernel]).

For the pipelined configs[1] steps: per consecutive pair of K1 launches (by start time) the idle gap between
them (negative: they overlap), K1's own duration, and which other kernels ran inside each gap.
"""
import csv
import sys
from collections import Counter

path = sys.argv[1]
kname = sys.argv[2] if len(sys.argv) > 2 else "k_replayable_sweep_oq"
rows = list(csv.DictReader(open(path)))
name_col = next(c for c in rows[0] if c.lower() in ("kernel_name", "name"))
st_col = next(c for c in rows[0] if "start" in c.lower())
en_col = next(c for c in rows[0] if "end" in c.lower())
ks = sorted((int(r[st_col]), int(r[en_col]), r[name_col]) for r in rows)
k1 = [k for k in ks if kname in k[2]]
k1 = k1[len(k1) // 3:]  # steady state: skip warm-up and the first steps
durs = [(e - s) / 1e3 for s, e, _ in k1]
gaps = []
inside = Counter()
for (s0, e0, _), (s1, e1, _) in zip(k1, k1[1:]):
    gaps.append((s1 - e0) / 1e3)
    for s, e, n in ks:
        if s < s1 and e > e0 and kname not in n:
            inside[n.split("(")[0][:48]] += 1
span = (k1[-1][1] - k1[0][0]) / 1e3
print(f"{len(k1)} K1 launches, {span:.1f} us from first start to last end = {span / len(k1):.2f} us per launch")
print(f"K1 duration: mean {sum(durs) / len(durs):.1f} min {min(durs):.1f} max {max(durs):.1f} us")
print(f"gap to the next K1 start: mean {sum(gaps) / len(gaps):.1f} min {min(gaps):.1f} max {max(gaps):.1f} us")
print("kernels overlapping the gaps:", dict(inside.most_common(8)))
