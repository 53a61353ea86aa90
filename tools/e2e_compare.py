#!/usr/bin/env python3
"""Python-driven trace stream vs the native batch call (nmz_replayable_sweep_traces) on one GPU timeline
(measurement tooling). Reads a rocprofv3 --kernel-trace --memory-copy-trace database of
`bench.py --legs replayable` and splits the plan-kernel launches into runs of T consecutive builds: the last run
is the last native batch call, the fourth from the end the native warm-up call, the fifth the timed Python stream
(the bench makes the timed stream, then a warm-up and three timed native calls). Prints, per run: span, busy
time, per-kernel totals and the streams used.

usage: python tools/e2e_compare.py gpurun_out/<dir> [T=64]
"""
import collections
import glob
import sqlite3
import sys


def run_stats(ev, s0, s1, T):
    seg = [e for e in ev if s0 <= e[0] < s1]
    busy, cur = 0, None
    for e in seg:
        if cur is None or e[0] > cur[1]:
            if cur:
                busy += cur[1] - cur[0]
            cur = [e[0], e[1]]
        else:
            cur[1] = max(cur[1], e[1])
    if cur:
        busy += cur[1] - cur[0]
    per = collections.defaultdict(lambda: [0, 0.0])
    streams = collections.Counter()
    for e in seg:
        per[e[2]][0] += 1
        per[e[2]][1] += (e[1] - e[0]) / 1e3
        streams[e[3]] += 1
    span = (s1 - s0) / 1e6
    print(f"  span {span:.3f} ms = {span / (T - 1):.4f} ms per trace; GPU busy {busy / 1e6:.3f} ms "
          f"({busy / (s1 - s0):.2f}); streams {dict(streams)}")
    for k, (n, us) in sorted(per.items(), key=lambda kv: -kv[1][1])[:10]:
        print(f"    {k:42s} {n:5d} launches {us / (T - 1):8.1f} us per trace")


def main():
    db = glob.glob(sys.argv[1] + "/**/*.db", recursive=True)[0]
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    c = sqlite3.connect(db)
    ev = [(r[1], r[2], r[0].split("(")[0][-40:], r[3]) for r in c.execute("select name,start,end,stream_id from kernels")]
    ev += [(r[0], r[1], "COPY %s" % r[4][-14:], r[3])
           for r in c.execute("select start,end,size,stream_id,name from memory_copies")]
    ev.sort()
    idx = [i for i, e in enumerate(ev) if "wt_build" in e[2]]
    print(f"{len(idx)} plan-kernel launches")
    for name, k in (("python stream (timed)", 5), ("native batch (warm-up call)", 4), ("native batch (last call)", 1)):
        first, last = idx[-k * T], idx[-(k - 1) * T - 1]
        print(name)
        run_stats(ev, ev[first][0], ev[last][0], T)


if __name__ == "__main__":
    main()
