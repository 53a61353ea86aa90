#!/usr/bin/env python3
"""Print per-kernel average durations from a rocprofv3 kernel_stats.csv (usage: kstats.py <csv> [filter])."""
import csv
import sys

flt = sys.argv[2] if len(sys.argv) > 2 else ""
for r in csv.DictReader(open(sys.argv[1])):
    if flt in r["Name"]:
        print(f"{r['Name'][:64]:64s} {r['Calls']:>4} {float(r['AverageNs']) / 1e3:10.1f} us")
