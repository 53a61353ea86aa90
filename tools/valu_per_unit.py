#!/usr/bin/env python3
"""Per-unit VALU lane-instruction counts from per-leg rocprofv3 summaries (tools/profile_r02.sh output).

usage: valu_per_unit.py <profile dir with one sub-directory per bench leg> <tag>
  -> profiles/valu_per_unit.json, which bench.py reads for each leg's roofline:
     ops_per_unit = SQ_INSTS_VALU x 64 / units per launch of that leg's workload,
     hbm_bytes_per_launch = 2 x FETCH_SIZE + WRITE_SIZE (gfx950 FETCH_SIZE correction),
     clock_ghz = GRBM_GUI_ACTIVE / 8 XCDs / duration.
The ED kernels' counts depend on the data through the cut-off, so each configs[2] generator has its own key.
"""
import json
import os
import sys

# leg -> [(kernel name prefix, key, unit, units per launch of the leg's default workload)]
LEGS = {
    # the order-query kernel (default) and the per-decision sweep (NMZ_REPLAY_OQ=0 runs of the same leg)
    "replayable": [("void nmz::k_replayable_sweep_wt<false", "k_replayable_sweep_wt", "decision", 2**20 * 4096),
                   ("void nmz::k_replayable_sweep_oq<false, false>", "k_replayable_sweep_oq", "decision", 2**20 * 4096),
                   ("void nmz::k_replayable_sweep_fast", "k_replayable_sweep_fast", "decision", 2**20 * 4096)],
    "random": [("void nmz::k_random_sweep", "k_random_sweep", "decision", 10_000_000 * 10_000)],
    # two-phase search: the DP kernel per pair that ran the DP (the k_ed_bv counters of the bench workload:
    # 51,032,886 clustered, 306,187 survey), the filter passes (count + write, one key) per pair of the search
    # the filter phase is the count pass plus the scatter (write) pass: bench.py times both under one name
    "ed_clustered": [("void nmz::k_ed_bv_dp<32, false>", "k_ed_bv_dp:clustered", "DP pair", 51_032_886),
                     ("void nmz::k_ed_qg_filter<", "k_ed_qg_filter:clustered", "pair", 100_000 * 99_999 // 2),
                     ("nmz::k_ed_qg_scatter", "k_ed_qg_filter:clustered", "pair", 100_000 * 99_999 // 2)],
    "ed_survey": [("void nmz::k_ed_bv_dp<32, false>", "k_ed_bv_dp:survey", "DP pair", 306_187),
                  ("void nmz::k_ed_qg_filter<", "k_ed_qg_filter:survey", "pair", 100_000 * 99_999 // 2),
                  ("nmz::k_ed_qg_scatter", "k_ed_qg_filter:survey", "pair", 100_000 * 99_999 // 2)],
    # compact tables (a store-wide alphabet of thousands of events): the CMP instantiation
    "ed_alphabet": [("void nmz::k_ed_bv_dp<32, true>", "k_ed_bv_dp:alphabet", "DP pair", 51_031_728),
                    ("void nmz::k_ed_qg_filter<", "k_ed_qg_filter:alphabet", "pair", 100_000 * 99_999 // 2),
                    ("nmz::k_ed_qg_scatter", "k_ed_qg_filter:alphabet", "pair", 100_000 * 99_999 // 2)],
    "ed_wide": [("void nmz::k_ed_wide<4>", "k_ed_wide", "pair", 256 * 255 // 2)],
    # one launch per mode per step (PO first, then exact): the profile's average mixes both modes, so the
    # per-mode figures come from the two kernel instantiations
    "visualize": [("void nmz::k_trace_sig<2>", "k_trace_sig:po", "trace", 100_000),
                  ("void nmz::k_trace_sig<0>", "k_trace_sig:exact", "trace", 100_000)],
}


def dp_pairs_of_run(leg_dir):
    """DP pairs of the profiled run's own search (bench JSON line on stdout: trace.json), or None."""
    # bench.py prints each secondary leg on its own line ({"secondary_leg": ...}) before the compact headline
    # (older runs: one line with a "secondary" list)
    try:
        lines = [json.loads(x) for x in open(os.path.join(leg_dir, "trace.json")).read().strip().splitlines()
                 if x.startswith("{")]
    except (OSError, ValueError):
        return None
    legs = [x["secondary_leg"] for x in lines if "secondary_leg" in x]
    for x in lines:
        legs += x.get("secondary", []) if isinstance(x.get("secondary"), list) else []
    for sec in legs:
        if sec.get("search", {}).get("dp_pairs"):
            return int(sec["search"]["dp_pairs"])
    return None


def main():
    src, tag = sys.argv[1], sys.argv[2]
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    import kernel_isa
    path = os.path.join(here, "..", "profiles", "valu_per_unit.json")
    out = json.load(open(path)) if os.path.exists(path) else {}
    # machine-code fingerprints of the library the profile ran (written on the box by tools/profile_r03.sh)
    isa_path = os.path.join(src, "isa.json")
    fps = json.load(open(isa_path)) if os.path.exists(isa_path) else kernel_isa.kernel_fingerprints()
    for leg, kernels in LEGS.items():
        f = os.path.join(src, leg, "summary.json")
        if not os.path.exists(f):
            continue
        summ = json.load(open(f))
        dp_run = dp_pairs_of_run(os.path.join(src, leg))
        seen = set()
        for name, e in sorted(summ.items()):
            for pre, key, unit, n in kernels:
                if unit == "DP pair" and dp_run:
                    n = dp_run
                if name.startswith(pre) and "SQ_INSTS_VALU" in e:
                    if key in seen:  # several kernels under one key (the filter's count and write passes): sum
                        o = out[key]
                        o["ops_per_unit"] += e["SQ_INSTS_VALU"] * 64 / n
                        o["avg_ns"] += e["avg_ns"]
                        if o.get("grbm") is not None and e.get("GRBM_GUI_ACTIVE") is not None:
                            # the clock over all of the key's kernels, weighted by their time
                            o["grbm"] += e["GRBM_GUI_ACTIVE"]
                            o["clock_ghz"] = o["grbm"] / 8 / o["avg_ns"]
                        o["kernel"] += " + " + name
                        o["isa"][name] = kernel_isa.lookup(fps, name)
                        if o.get("hbm_bytes_per_launch") is not None and e.get("hbm_bytes_fetch_x2") is not None:
                            o["hbm_bytes_per_launch"] += e["hbm_bytes_fetch_x2"]
                        continue
                    seen.add(key)
                    out[key] = {"ops_per_unit": e["SQ_INSTS_VALU"] * 64 / n, "unit": unit, "units_per_launch": n,
                                "kernel": name, "avg_ns": e["avg_ns"],
                                "source": f"SQ_INSTS_VALU per launch, profiles/{tag}_{leg}_summary.json",
                                "hbm_bytes_per_launch": e.get("hbm_bytes_fetch_x2"),
                                "clock_ghz": e.get("clock_ghz"), "grbm": e.get("GRBM_GUI_ACTIVE"),
                                # fingerprints of the profiled kernels (tools/kernel_isa.py): bench.py marks the
                                # entry stale when the shipped library's kernels differ
                                "isa": {name: kernel_isa.lookup(fps, name)}}
    json.dump(out, open(path, "w"), indent=1, sort_keys=True)
    for k, v in sorted(out.items()):
        print(f"{k:26s} {v['ops_per_unit']:14.3f} VALU lane-instr / {v['unit']}  ({v['source']})")


if __name__ == "__main__":
    main()
