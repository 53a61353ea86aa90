#!/usr/bin/env python3
"""Summarize a rocprofv3 run directory (kernel stats + PMC passes) into JSON.

usage: summarize_profile.py <prof_dir> <out.json>
FETCH_SIZE / WRITE_SIZE are in KiB per dispatch; gfx950 FETCH_SIZE under-counts
wide streaming reads by 2x (MI355X_MICROARCH.md, HBM) -- the raw value is kept
and the streaming-corrected upper bound is reported beside it.
GRBM_GUI_ACTIVE is summed over the 8 XCDs.
"""
import collections
import csv
import json
import os
import sys


def agg(path):
    d = collections.defaultdict(lambda: collections.defaultdict(list))
    if not os.path.exists(path):
        return d
    for r in csv.DictReader(open(path)):
        d[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return d


def main():
    src, out = sys.argv[1], sys.argv[2]
    stats = {r["Name"]: r for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv")))}
    v = agg(os.path.join(src, "pmc_valu", "run_counter_collection.csv"))
    f = agg(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    w = agg(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    res = {}
    for name, r in stats.items():
        e = {"calls": int(r["Calls"]), "avg_ns": float(r["AverageNs"]), "pct": float(r["Percentage"])}
        for d in (v, f, w):
            for c, vals in d.get(name, {}).items():
                e[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in e and "WRITE_SIZE" in e:
            e["hbm_bytes_raw"] = (e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
            e["hbm_bytes_fetch_x2"] = (2 * e["FETCH_SIZE"] + e["WRITE_SIZE"]) * 1024
        if "GRBM_GUI_ACTIVE" in e and e["avg_ns"] > 0:
            e["clock_ghz"] = e["GRBM_GUI_ACTIVE"] / 8 / e["avg_ns"]
        res[name] = e
    json.dump(res, open(out, "w"), indent=1, sort_keys=True)
    for n, e in sorted(res.items(), key=lambda t: -t[1]["pct"]):
        print(f"{e['pct']:6.2f}% {e['avg_ns']/1e3:10.1f} us x{e['calls']:3d}  {n[:70]}")


if __name__ == "__main__":
    main()
