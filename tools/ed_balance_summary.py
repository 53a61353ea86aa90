#!/usr/bin/env python3
"""Summarise tools/ed_shard_balance.py records: per file, unsharded ms, max / sum of shards, bound, shard filter / DP."""
import glob
import json
import sys

for f in sorted(glob.glob(sys.argv[1])):
    d = json.load(open(f))
    ps = d["per_shard"]
    print(f"{f.split('/')[-1]:48s} unsharded {d['unsharded_ms']:8.3f}  max {d['max_shard_ms']:7.3f}  "
          f"sum/unsh {d['sum_shard_ms'] / d['unsharded_ms']:.3f}  bound {d['speedup_bound']:.3f}  "
          f"filter {max(p['filter_ms'] for p in ps):.3f}  dp {max(p['dp_ms'] for p in ps):.3f}"
          + (f"  | uninstrumented: unsharded {d['uninstrumented']['unsharded_ms']:.3f}  max "
             f"{d['uninstrumented']['max_shard_ms']:.3f}  sum/unsh {d['uninstrumented']['sum_over_unsharded']:.3f}  "
             f"bound {d['uninstrumented']['speedup_bound']:.3f}" if "uninstrumented" in d else ""))
