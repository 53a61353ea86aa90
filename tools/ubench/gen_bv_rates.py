#!/usr/bin/env python3
"""Generate tools/ubench/bv_rates.hip: issue cost of the VALU forms a
bit-parallel (Myers/Hyyro) edit-distance column step uses on gfx950.
Each kernel runs 8 independent chains of one instruction form; cycles per
wave64 instruction per SIMD = clock64 delta / (iters * 32) at 8 waves/SIMD."""
FORMS = [
    ("bitop3_vvv", "v_bitop3_b32 {d}, {d}, %[a], %[b] bitop3:0xf1"),
    ("alignbit_vvv", "v_alignbit_b32 {d}, {d}, %[a], %[b]"),
    ("alignbit_vvs", "v_alignbit_b32 {d}, {d}, %[a], %[sg]"),
    ("alignbit_vvi", "v_alignbit_b32 {d}, {d}, %[a], 1"),
    ("add_co", "v_add_co_u32 {d}, vcc, {d}, %[a]"),
    ("addc_co", "v_addc_co_u32 {d}, vcc, {d}, %[a], vcc"),
    ("bcnt", "v_bcnt_u32_b32 {d}, {d}, %[a]"),
    ("and_or", "v_and_or_b32 {d}, {d}, %[a], %[b]"),
    ("or_vv", "v_or_b32 {d}, {d}, %[a]"),
    ("lshrrev_vs", "v_lshrrev_b32 {d}, %[sg], {d}"),
    ("add_vs", "v_add_u32 {d}, %[sg], {d}"),
    ("lshl_add_u64", "v_lshl_add_u64 {w}, {w}, 0, %[wa]"),
    # forms of the issue-ceiling mixes (tools/issue_ceiling.py)
    ("lshrrev_vv", "v_lshrrev_b32 {d}, %[a], {d}"),
    ("lshrrev_vi", "v_lshrrev_b32 {d}, 3, {d}"),
    ("xor_vi", "v_xor_b32 {d}, 1, {d}"),
    ("xor_vv", "v_xor_b32 {d}, %[a], {d}"),
    ("add3", "v_add3_u32 {d}, {d}, %[a], %[b]"),
    ("lshl_add_u32", "v_lshl_add_u32 {d}, {d}, 2, %[a]"),
    ("bfe_vvv", "v_bfe_u32 {d}, {d}, %[a], %[b]"),
    ("bcnt_vi", "v_bcnt_u32_b32 {d}, {d}, 0"),
    ("cndmask_vcc", "v_cndmask_b32 {d}, {d}, %[a], vcc"),
    ("cndmask_e64_s", "v_cndmask_b32_e64 {d}, {d}, %[a], %[sm]"),
    ("min_u32", "v_min_u32 {d}, {d}, %[a]"),
    ("mul_hi_u32", "v_mul_hi_u32 {d}, {d}, %[a]"),
    ("mul_u24", "v_mul_u32_u24 {d}, {d}, %[a]"),
    ("mad_u64_u32", "v_mad_u64_u32 {w}, vcc, %[a], %[b], {w}"),
    ("cmp_lt_e32", "v_cmp_lt_u32 vcc, {d}, %[a]"),
    ("mov_dpp", "v_mov_b32_dpp {d}, {d} row_shr:1"),
    ("subrev_co", "v_subrev_co_u32 {d}, vcc, {d}, %[a]"),
    ("mov_vv", "v_mov_b32 {d}, %[a]"),
    ("bitop3_vvi", "v_bitop3_b32 {d}, {d}, %[a], 5 bitop3:0xf1"),
    # the q-gram filter and its scatter (k_ed_qg_filter / k_ed_qg_scatter): SAD accumulation chains, the
    # SGPR-operand form, and the lane-prefix count of the entry scatter
    ("sad_u8_vvv", "v_sad_u8 {d}, %[a], %[b], {d}"),
    ("sad_u8_vsv", "v_sad_u8 {d}, %[a], %[sg], {d}"),
    ("mbcnt_lo", "v_mbcnt_lo_u32_b32 {d}, %[a], {d}"),
    ("mbcnt_hi", "v_mbcnt_hi_u32_b32 {d}, %[a], {d}"),
]
ITERS = 4096
out = ['#include <hip/hip_runtime.h>', '#include <cstdio>', '#include <cstdint>', f'#define ITERS {ITERS}']
for n, (name, form) in enumerate(FORMS):
    body = []
    for rep in range(4):
        for r in range(8):
            body.append(form.format(d=f"%{r}", w=f"%[w{r}]"))
    asm = "\\n\\t".join(body)
    out.append(f'''__global__ __launch_bounds__(256) void k{n}(uint32_t* out, uint64_t* clk, uint32_t seed) {{
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {{
    asm volatile("{asm}" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }}
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[{n}] = t1 - t0;
}}''')
launches = "\n".join(
    f'  hipLaunchKernelGGL(k{n}, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); '
    f'hipLaunchKernelGGL(k{n}, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); '
    f'hipEventSynchronize(e1); hipEventElapsedTime(&ms[{n}], e0, e1);'
    for n in range(len(FORMS)))
names = ", ".join(f'"{f[0]}"' for f in FORMS)
out.append(f'''int main() {{
  const int blocks = 256 * 8;  // 8 waves per SIMD
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms[64];
  uint32_t* out; uint64_t* clk; hipMalloc(&out, blocks * 256 * 4); hipMallocManaged(&clk, 64 * 8);
{launches}
  const char* names[] = {{{names}}};
  for (int n = 0; n < {len(FORMS)}; ++n)
    printf("%-14s %.3f ms  %.2f cyc@2.4GHz per wave-instr per SIMD  (clock64 %.2f)\\n", names[n], ms[n], ms[n] * 1e-3 * 2.4e9 / ({ITERS} * 32.0 * 8.0), (double)clk[n] / ({ITERS} * 32.0));
  return 0;
}}''')
open(__file__.replace("gen_bv_rates.py", "bv_rates.hip"), "w").write("\n".join(out) + "\n")
