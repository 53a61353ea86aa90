#!/usr/bin/env python3
"""GPU timeline of bench.py's timed headline region (configs[1]) from a rocprofv3 --kernel-trace database
(measurement tooling): the region is the last `steps` seed-prefix launches before the job merge's last launch, up to
that merge's end. Prints the region's span, per-step kernel intervals per stream, per-kernel totals and the CU-idle
gaps (no kernel running), so fill, drain and launch gaps are visible.

usage: python tools/headline_timeline.py gpurun_out/<dir> [steps=20]
"""
import collections
import glob
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    c = sqlite3.connect(db)
    ev = sorted((r[1], r[2], r[0].split("(")[0].replace("void ", "")[-34:], r[3])
                for r in c.execute("select name,start,end,stream_id from kernels"))
    merges = [i for i, e in enumerate(ev) if "topk_merge" in e[2]]
    m = merges[-1]
    pre = [i for i, e in enumerate(ev[:m]) if "seed_prefix" in e[2]][-steps:]
    t0, t1 = ev[pre[0]][0], ev[m][1]
    seg = [e for e in ev[pre[0]:m + 1]]
    print("timed region (first seed prefix start -> job merge end): %.1f us = %.2f us per step"
          % ((t1 - t0) / 1e3, (t1 - t0) / 1e3 / steps))
    k1 = [e for e in seg if "sweep_wt" in e[2]]
    print("K1: %d launches, first start %.1f us, last end %.1f us, avg duration %.1f us"
          % (len(k1), (k1[0][0] - t0) / 1e3, (k1[-1][1] - t0) / 1e3,
             sum(e[1] - e[0] for e in k1) / len(k1) / 1e3))
    if len(k1) > 1:
        st = [(b[0] - a[0]) / 1e3 for a, b in zip(k1, k1[1:])]
        print("K1 start-to-start: " + " ".join("%.1f" % x for x in st))
        ov = [(b[0] - a[1]) / 1e3 for a, b in zip(k1, k1[1:])]
        print("K1 end-to-next-start (negative = overlap): " + " ".join("%.1f" % x for x in ov))
    tot = collections.defaultdict(lambda: [0, 0])
    for e in seg:
        tot[e[2]][0] += 1
        tot[e[2]][1] += e[1] - e[0]
    for k, v in sorted(tot.items(), key=lambda x: -x[1][1]):
        print("  %-36s %3d  %8.1f us avg  %8.1f us total" % (k, v[0], v[1] / v[0] / 1e3, v[1] / 1e3))
    busy, cur, gaps = 0, None, []
    for e in seg:
        if cur is None or e[0] > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
                gaps.append(((e[0] - cur[1]) / 1e3, e[2], (e[0] - t0) / 1e3))
            cur = [e[0], e[1]]
        else:
            cur[1] = max(cur[1], e[1])
    busy += cur[1] - cur[0]
    print("busy %.1f us; idle gaps %d totalling %.1f us; largest:" % (busy / 1e3, len(gaps),
                                                                       sum(g[0] for g in gaps)))
    for g in sorted(gaps, reverse=True)[:8]:
        print("   %.1f us before %s at %.1f us" % g)
    print("--- first and last 40 ops (us from region start)")
    for e in seg[:40] + [None] + seg[-40:]:
        if e is None:
            print("   ...")
            continue
        print("%8.1f %8.1f  s%-3d %s" % ((e[0] - t0) / 1e3, (e[1] - t0) / 1e3, e[3], e[2]))


if __name__ == "__main__":
    main()
