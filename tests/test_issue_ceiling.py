"""The issue-cost ceiling tool (tools/issue_ceiling.py): its per-form prices follow the ubench measurements
(profiles/r03ub_issue_rates.log), and its hot-loop pricing of the shipped library is what bench.py reports."""
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "tools"))
import issue_ceiling as IC  # noqa: E402


@pytest.mark.parametrize("mn,ops,cls,cost", [
    ("v_xor_b32_e32", "v1, v2, v3", "full", IC.COST_FULL),          # VGPR-only VOP2
    ("v_lshrrev_b32_e32", "v1, 3, v2", "full", IC.COST_FULL),       # inline constant: measured full rate (2.15)
    ("v_add_co_u32_e32", "v1, vcc, v2, v3", "full", IC.COST_FULL),  # VCC carry form
    ("v_add_u32_e32", "v1, s4, v2", "half", IC.COST_HALF),          # SGPR operand
    ("v_add_u32_e32", "v1, 0x12345678, v2", "half", IC.COST_HALF),  # 32-bit literal
    ("v_cndmask_b32_e64", "v1, v2, v3, s[0:1]", "half", IC.COST_HALF),
    ("v_bcnt_u32_b32", "v1, v2, v3", "half", IC.COST_HALF),
    ("v_cmp_lt_u32_e32", "vcc, v1, v2", "half", IC.COST_HALF),
    ("v_bitop3_b32", "v1, v2, v3, v4 bitop3:0xf1", "full", 2.8),
    ("v_alignbit_b32", "v1, v2, v3, 1", "half", 4.4),
    ("v_mad_u64_u32", "v[0:1], s[0:1], v2, v3, v[4:5]", "half", 4.2),
    ("v_exp_f32_e32", "v1, v2", "trans", IC.COST_TRANS),
])
def test_classify_follows_measured_costs(mn, ops, cls, cost):
    assert IC.classify(mn, ops) == (cls, cost)


def test_mix_counts_and_mean():
    ins = [(0, "v_xor_b32_e32", "v1, v2, v3", None), (4, "v_add_u32_e32", "v1, s4, v2", None),
           (8, "ds_read_b64", "v[0:1], v2", None), (12, "s_add_i32", "s1, s1, 1", None),
           (16, "s_waitcnt", "lgkmcnt(0)", None)]
    m = IC.mix(ins)
    assert (m["full"], m["half"], m["lds"], m["salu"], m["valu"]) == (1, 1, 1, 1, 2)
    assert m["mean_cost"] == pytest.approx((IC.COST_FULL + IC.COST_HALF) / 2)


def test_hot_loop_is_the_innermost_loop_with_most_valu():
    # outer loop [0, 40] holds inner loops [8, 16] (1 VALU) and [20, 36] (3 VALU)
    ins = [(0, "v_mov_b32_e32", "v0, v1", None), (8, "v_add_u32_e32", "v0, v0, v1", None),
           (16, "s_cbranch_scc1", "", 8), (20, "v_xor_b32_e32", "v0, v0, v1", None),
           (24, "v_xor_b32_e32", "v0, v0, v1", None), (28, "v_xor_b32_e32", "v0, v0, v1", None),
           (36, "s_cbranch_vccnz", "", 20), (40, "s_branch", "", 0)]
    s, e, body = IC.hot_loop(ins)
    assert (s, e) == (20, 36) and sum(1 for x in body if x[1].startswith("v_")) == 3


def test_committed_ceilings_match_the_library():
    """profiles/issue_ceiling.json prices kernels whose machine code is the shipped library's (the bench reports
    frac_of_issue_ceiling only then), and K2 sits at its ceiling."""
    lib = os.path.join(HERE, "..", "namazu_amd", "libnmz_gpu.so")
    if not os.path.exists(lib) or not os.path.exists(IC.OBJDUMP):
        pytest.skip("library or llvm-objdump missing")
    import kernel_isa
    fps = kernel_isa.kernel_fingerprints(lib)
    d = json.load(open(os.path.join(HERE, "..", "profiles", "issue_ceiling.json")))["kernels"]
    assert {"k_random_sweep", "k_ed_bv_dp:clustered", "k_ed_wide", "k_replayable_sweep_wt"} <= set(d)
    for e in d.values():
        assert e["isa"] and 0.3 < e["hot_loop"]["at_ceiling"] < 1.1
    stale = [n for n, e in d.items() if any(kernel_isa.lookup(fps, k) != h for k, h in e["isa"].items())]
    if stale:  # bench.py then reports no frac_of_issue_ceiling for them
        pytest.skip(f"kernels changed since their profile (re-profile, then tools/issue_ceiling.py): {stale}")
    assert d["k_random_sweep"]["hot_loop"]["at_ceiling"] > 0.95
