#!/usr/bin/env python3
"""GPU timeline of bench.py's streamed end-to-end traces from a rocprofv3 --kernel-trace --memory-copy-trace
database (measurement tooling): per-trace span and busy time over the last 17 plan-kernel launches, per-kernel
totals, the largest gaps, and the ops around one plan kernel.

usage: python tools/e2e_timeline.py gpurun_out/<dir>  [n_traces=17]
"""
import collections
import glob
import sqlite3
import sys


def main():
    db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 17
    c = sqlite3.connect(db)
    ev = [(r[1], r[2], r[0].split("(")[0][-40:], r[3]) for r in c.execute("select name,start,end,stream_id from kernels")]
    ev += [(r[0], r[1], "COPY %s %d" % (r[4][-14:], r[2]), r[3])
           for r in c.execute("select start,end,size,stream_id,name from memory_copies")]
    ev.sort()
    idx = [i for i, e in enumerate(ev) if "wt_build" in e[2]]
    s0, s1 = ev[idx[-T]][0], ev[idx[-1]][0]
    seg = [e for e in ev if s0 <= e[0] < s1]
    busy, cur, gaps = 0, None, []
    for e in seg:
        if cur is None or e[0] > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
                gaps.append((e[0] - cur[1], e[2], (e[0] - s0) / 1e6))
            cur = [e[0], e[1]]
        else:
            cur[1] = max(cur[1], e[1])
    busy += cur[1] - cur[0]
    n = T - 1
    print("%d traces: span %.3f ms, busy %.3f ms; per trace span %.1f us, busy %.1f us"
          % (n, (s1 - s0) / 1e6, busy / 1e6, (s1 - s0) / n / 1e3, busy / n / 1e3))
    tot = collections.defaultdict(lambda: [0, 0, 0])
    for e in seg:
        tot[e[2]][0] += 1
        tot[e[2]][1] += e[1] - e[0]
        tot[e[2]][2] = max(tot[e[2]][2], e[1] - e[0])
    for k, v in sorted(tot.items(), key=lambda x: -x[1][1]):
        print("%-42s %4d  %7.1f us/trace  %7.1f us avg  %8.1f us max" % (k, v[0], v[1] / n / 1e3, v[1] / v[0] / 1e3,
                                                                        v[2] / 1e3))
    print("largest GPU-idle gaps (us, next op, at ms):",
          [(round(g / 1e3, 1), nm, round(t, 2)) for g, nm, t in sorted(gaps, reverse=True)[:5]])
    a = ev[idx[-5]][0]
    print("--- ops around a plan kernel (us from its start)")
    for e in ev:
        if a - 60000 <= e[0] < a + 260000:
            print("%8.1f %8.1f  s%-3d %s" % ((e[0] - a) / 1e3, (e[1] - a) / 1e3, e[3], e[2]))


if __name__ == "__main__":
    main()
