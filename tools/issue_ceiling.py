#!/usr/bin/env python3
"""VALU issue-cost ceilings of the integer kernels (measurement infrastructure, not the product).

For each kernel priced in profiles/valu_per_unit.json this prices its instruction mix with the gfx950 issue costs
that tools/ubench measured, and compares the resulting lower bound on the kernel's duration with the
measured one:

  * the dynamic count: SQ_INSTS_VALU wave-instructions per launch (valu_per_unit.json: lane-instructions per unit x
    units per launch / 64, from a HEAD rocprofv3 pass; the entry's machine-code fingerprint must match the library);
  * the mix: the hot loop's static gfx950 code (llvm-objdump of the kernel inside libnmz_gpu.so), each VALU
    instruction priced by `classify` with the costs tools/ubench/bv_rates.hip measured (profiles/r03ub_issue_rates.log,
    cycles per wave64 instruction per SIMD at 8 waves/SIMD): VOP1/VOP2 forms with VGPR, inline-constant or VCC
    operands ~2.2; VOP3 forms, compares, SGPR / literal operands, 32-bit min/max, multiplies, bcnt/bfe/add3,
    packed and DPP forms ~4.1; v_bitop3 2.8, v_alignbit 4.4, v_lshl_add_u64 4.35, v_mad_u64_u32 4.2;
  * the ceiling: count x mean cost / (1,024 SIMDs x the clock the chip held in that launch, GRBM_GUI_ACTIVE / 8 /
    duration). `at_ceiling` = ceiling / measured duration: 1.0 means the SIMDs issued VALU every cycle at this mix.

The hot loop is the innermost loop (a backward branch with no other backward branch inside) holding the most VALU
instructions; the whole kernel's static code is priced too (`whole_kernel`). Both are printed. A VOP2 carry or
select form is priced at full rate, which is what it costs when its VCC producer is adjacent; the
ceiling is a lower bound on the duration, so `at_ceiling` can only be overstated by such optimistic prices.

usage: issue_ceiling.py [--lib libnmz_gpu.so] [--out profiles/issue_ceiling.json]
(bench.py reads profiles/issue_ceiling.json: `frac_of_issue_ceiling` in a leg's roofline, when the kernel's
fingerprint there matches the shipped library)
"""
import argparse
import json
import os
import re
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import kernel_isa  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"
COST_FULL, COST_HALF, COST_TRANS = 2.2, 4.1, 8.0
SIMDS = 256 * 4

# kernel entry in valu_per_unit.json -> mangled symbol prefix
KERNELS = {
    "k_replayable_sweep_wt": "_ZN3nmz21k_replayable_sweep_wtILb0ELi1ELi6E",
    "k_random_sweep": "_ZN3nmz14k_random_sweepILb1E",
    "k_ed_bv_dp:clustered": "_ZN3nmz10k_ed_bv_dpILi32ELb0E",
    "k_ed_bv_dp:alphabet": "_ZN3nmz10k_ed_bv_dpILi32ELb1E",
    "k_ed_wide": "_ZN3nmz9k_ed_wideILi4E",
    # the q-gram filter's key holds its count and scatter passes (one timer in bench.py); the count pass's hot loop
    # (v_sad_u8, measured at 4.10 cycles: profiles/r04/r04ub_issue_rates.log) prices both
    "k_ed_qg_filter:survey": "_ZN3nmz14k_ed_qg_filterILb1E",
    "k_ed_qg_filter:clustered": "_ZN3nmz14k_ed_qg_filterILb1E",
    # visualize: one wave per trace, 64 elements per step (PO: entity ballots + LDS rank counters + the mix)
    "k_trace_sig:po": "_ZN3nmz11k_trace_sigILi2E",
    "k_trace_sig:exact": "_ZN3nmz11k_trace_sigILi0E",
}

# cycles per wave64 instruction per SIMD at 8 waves/SIMD, tools/ubench/bv_rates.hip (profiles/r03ub_issue_rates.log)
FORM_COST = {"v_bitop3_b32": 2.8, "v_alignbit_b32": 4.4, "v_lshl_add_u64": 4.35, "v_mad_u64_u32": 4.2,
             "v_sad_u8": 4.10}
HALF_OPS = ("v_min_u32", "v_max_u32", "v_min_i32", "v_max_i32", "v_readfirstlane", "v_cmp", "v_cmpx", "v_mul",
            "v_mad", "v_bcnt", "v_mbcnt", "v_bfe", "v_bfi", "v_add3", "v_lshl_add", "v_lshl_or", "v_and_or", "v_or3",
            "v_xor3", "v_xad", "v_perm", "v_readlane", "v_writelane", "v_lshlrev_b64", "v_lshrrev_b64")
TRANS_OPS = ("v_exp", "v_log", "v_rcp", "v_rsq", "v_sqrt", "v_sin", "v_cos")
INLINE = re.compile(r"^-?(\d+|0x[0-9a-f]+)$")


def classify(mn, ops):
    """(class, cycles) of one VALU instruction (mnemonic, operand string) under the measured gfx950 costs:
    VOP1/VOP2 forms with VGPR, inline-constant or VCC (carry / select mask) operands are full rate; SGPR or
    32-bit literal operands, VOP3 / VOP3P / DPP / SDWA forms, compares and the ops listed in HALF_OPS are half rate;
    FORM_COST overrides both for the forms measured on their own."""
    base = mn[:-4] if mn.endswith(("_e32", "_e64")) else mn
    if mn.startswith(TRANS_OPS):
        return "trans", COST_TRANS
    if base in FORM_COST:
        return ("full" if FORM_COST[base] < 3 else "half"), FORM_COST[base]
    if mn.endswith("_e64") or "_sdwa" in mn or "_dpp" in mn or "row_" in ops or "quad_perm" in ops \
            or mn.startswith(("v_pk_",) + HALF_OPS):
        return "half", COST_HALF
    for tok in re.split(r"[,\s]+", ops.strip()):
        if not tok or tok.startswith("vcc") or (tok.startswith("v") and not tok.startswith("vcc")):
            continue
        if INLINE.match(tok) and -16 <= int(tok, 0) <= 64:
            continue
        return "half", COST_HALF  # an SGPR, exec, m0 or 32-bit literal source
    return "full", COST_FULL


def disassemble(img, sym):
    with tempfile.NamedTemporaryFile(suffix=".o") as f:
        f.write(img)
        f.flush()
        out = subprocess.run([OBJDUMP, "-d", "--no-show-raw-insn", "--disassemble-symbols=" + sym, f.name],
                             capture_output=True, text=True, check=True).stdout
    ins = []
    for line in out.splitlines():
        m = re.match(r"\s+(\S+)\s*(.*?)\s*//\s*([0-9A-Fa-f]+):(.*)$", line)
        if not m:
            continue
        mn, ops, addr, rest = m.group(1), m.group(2), int(m.group(3), 16), m.group(4)
        tgt = None
        t = re.search(r"<[^>]*\+0x([0-9a-f]+)>", rest)
        if t and mn.startswith(("s_cbranch", "s_branch")):
            tgt = int(t.group(1), 16)
        ins.append((addr, mn, ops, tgt))
    base = ins[0][0] if ins else 0
    return [(a - base, mn, ops, tgt) for a, mn, ops, tgt in ins]


def mix(ins):
    c = {"full": 0, "half": 0, "trans": 0, "salu": 0, "lds": 0, "vmem": 0, "smem": 0}
    half_ops = {}
    cycles = 0.0
    for _, mn, ops, _ in ins:
        if mn.startswith("v_"):
            k, cost = classify(mn, ops)
            c[k] += 1
            cycles += cost
            if k == "half":
                half_ops[mn] = half_ops.get(mn, 0) + 1
        elif mn.startswith("ds_"):
            c["lds"] += 1
        elif mn.startswith(("global_", "buffer_", "flat_")):
            c["vmem"] += 1
        elif mn.startswith("s_load") or mn.startswith("s_buffer_load"):
            c["smem"] += 1
        elif mn.startswith("s_") and not mn.startswith(("s_waitcnt", "s_cbranch", "s_branch", "s_nop", "s_barrier",
                                                         "s_endpgm", "s_setprio", "s_sleep")):
            c["salu"] += 1
    nv = c["full"] + c["half"] + c["trans"]
    c["valu"] = nv
    c["mean_cost"] = cycles / nv if nv else 0.0
    c["half_share"] = c["half"] / nv if nv else 0.0
    c["top_half_forms"] = dict(sorted(half_ops.items(), key=lambda kv: -kv[1])[:8])
    return c


def hot_loop(ins):
    loops = []
    for i, (a, mn, _, tgt) in enumerate(ins):
        if tgt is not None and tgt <= a:
            loops.append((tgt, a))
    inner = [(s, e) for s, e in loops if not any(s <= s2 and e2 <= e and (s2, e2) != (s, e) for s2, e2 in loops)]
    best, best_n = None, -1
    for s, e in inner:
        body = [x for x in ins if s <= x[0] <= e]
        n = sum(1 for x in body if x[1].startswith("v_"))
        if n > best_n:
            best, best_n = (s, e, body), n
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", default=os.path.join(HERE, "..", "namazu_amd", "libnmz_gpu.so"))
    ap.add_argument("--vpu", default=os.path.join(HERE, "..", "profiles", "valu_per_unit.json"))
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    blob = open(a.lib, "rb").read()
    syms = {}
    for img in kernel_isa.code_objects(blob):
        for name, _ in kernel_isa.elf_symbols(img):
            if not name.endswith(".kd"):
                syms[name] = img
    vpu = json.load(open(a.vpu))
    fps = kernel_isa.kernel_fingerprints(a.lib)
    res = {}
    for key, prefix in KERNELS.items():
        e = vpu.get(key)
        sym = next((s for s in syms if s.startswith(prefix)), None)
        if e is None or sym is None:
            continue
        fresh = all(kernel_isa.lookup(fps, k) == h for k, h in e.get("isa", {}).items())
        ins = disassemble(syms[sym], sym)
        s, t, body = hot_loop(ins)
        lm, wm = mix(body), mix(ins)
        wave_instr = e["ops_per_unit"] * e["units_per_launch"] / 64.0
        ghz, ns = e["clock_ghz"], e["avg_ns"]
        r = {"kernel": e["kernel"], "profile": e["source"], "fingerprint_matches_library": fresh,
             "isa": e.get("isa", {}),
             "valu_wave_instr_per_launch": wave_instr, "avg_ns": ns, "clock_ghz": ghz,
             "hot_loop": {"bytes": [s, t], **lm}, "whole_kernel": wm}
        for tag, m in (("hot_loop", lm), ("whole_kernel", wm)):
            cyc = wave_instr * m["mean_cost"] / SIMDS
            r[tag]["ceiling_ns_at_held_clock"] = cyc / ghz
            r[tag]["at_ceiling"] = cyc / ghz / ns
        r["full_rate_only_at_ceiling"] = wave_instr * COST_FULL / SIMDS / ghz / ns
        res[key] = r
        print(f"{key:24s} fresh={fresh} VALU {wave_instr:.3e} wave-instr, {ns / 1e6:.3f} ms @ {ghz:.2f} GHz | "
              f"hot loop {lm['valu']} VALU, half {lm['half_share']:.2f}, mean {lm['mean_cost']:.2f} cyc -> "
              f"at_ceiling {r['hot_loop']['at_ceiling']:.3f} | whole half {wm['half_share']:.2f} -> "
              f"{r['whole_kernel']['at_ceiling']:.3f} | all-full {r['full_rate_only_at_ceiling']:.3f}")
    if a.out:
        json.dump({"costs_cycles_per_wave_instr": {"full": COST_FULL, "half": COST_HALF, "trans": COST_TRANS},
                   "simds": SIMDS, "kernels": res}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
