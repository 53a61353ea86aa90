#!/usr/bin/env python3
"""Per-unit VALU lane-instruction counts from a rocprofv3 summary (tools/summarize_profile.py output).

usage: valu_per_unit.py <summary.json> <tag>  -> writes profiles/valu_per_unit.json, which bench.py reads
for each kernel's roofline (ops_per_unit = SQ_INSTS_VALU * 64 / units per launch). Units per launch are
the bench workloads' (tools/profile.sh runs bench.py with its defaults).
"""
import json
import os
import sys

UNITS = {  # kernel name prefix -> (unit, units per launch of the bench workload)
    "void nmz::k_replayable_sweep_fast": ("decision", 2**20 * 4096),
    "nmz::k_random_sweep": ("decision", 2**20 * 10_000),
    "void nmz::k_random_sweep<true>": ("decision", 2**20 * 10_000),
    "void nmz::k_ed_bv<32>": ("pair", 100_000 * 99_999 // 2),
    "void nmz::k_ed_wide<4>": ("pair", 256 * 255 // 2),
}


def main():
    src, tag = sys.argv[1], sys.argv[2]
    summ = json.load(open(src))
    out = {}
    for name, e in summ.items():
        for pre, (unit, n) in UNITS.items():
            if name.startswith(pre) and "SQ_INSTS_VALU" in e:
                key = pre.split("::")[1].split("<")[0]
                out[key] = {"ops_per_unit": e["SQ_INSTS_VALU"] * 64 / n, "unit": unit, "units_per_launch": n,
                            "kernel": name, "source": f"SQ_INSTS_VALU per launch, profiles/{tag}_summary.json",
                            "hbm_bytes_per_launch": e.get("hbm_bytes_fetch_x2"),
                            "clock_ghz": e.get("clock_ghz")}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "profiles", "valu_per_unit.json")
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    for k, v in out.items():
        print(f"{k:24s} {v['ops_per_unit']:14.3f} VALU lane-instr / {v['unit']}")


if __name__ == "__main__":
    main()
