// VCC / lane-mask microbenchmark (gfx950). tools/ubench/vgpr_banks.hip found that a v_cndmask_b32
// reading a VCC written long before costs ~23.6 cycles per wave64 instruction per SIMD, while K1's
// v_sub_co (writes VCC) -> v_cndmask (reads it) pairs issue at ~2 cycles. This measures the pair
// with 0, 1 and 2 instructions or s_nop wait states between producer and consumer, the SGPR-pair
// (VOP3) forms, and a second consumer of the same VCC.
// Build: hipcc --offload-arch=gfx950 -O3 -o vcc_fwd vcc_fwd.hip ; run on the box.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 4096
#define R8(X) X X X X X X X X
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55"

#define KERNEL(NAME, PAT)                                                                                  \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                           \
        asm volatile("v_mov_b32 v40, %0\n\tv_add_u32 v41, 3, %0\n\tv_add_u32 v42, 5, %0\n\tv_mov_b32 v43, %0\n\t" \
                     "v_mov_b32 v44, %0\n\tv_mov_b32 v45, %0\n\tv_cmp_gt_u32 vcc, 17, %0\n\t"                 \
                     "s_mov_b64 s[20:21], vcc" ::"v"(seed + threadIdx.x)                                       \
                     : CLOB, "vcc", "s20", "s21");                                                           \
        for (int it = 0; it < ITERS; ++it) asm volatile(R8(PAT)::: CLOB, "vcc", "s20", "s21");              \
        uint32_t r;                                                                                          \
        asm volatile("v_xor_b32 %0, v48, v49" : "=v"(r)::CLOB);                                               \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                                            \
    }

// producer/consumer pair, adjacent (K1's form)
KERNEL(k_pair_adj, "v_sub_co_u32 v48, vcc, v41, v42\n\tv_cndmask_b32 v49, v48, v41, vcc\n\t"
                   "v_sub_co_u32 v50, vcc, v42, v41\n\tv_cndmask_b32 v51, v50, v42, vcc\n\t")
// one independent VOP2 between producer and consumer
KERNEL(k_pair_gap1, "v_sub_co_u32 v48, vcc, v41, v42\n\tv_add_u32 v52, v43, v44\n\tv_cndmask_b32 v49, v48, v41, vcc\n\t"
                    "v_sub_co_u32 v50, vcc, v42, v41\n\tv_add_u32 v53, v43, v44\n\tv_cndmask_b32 v51, v50, v42, vcc\n\t")
// s_nop 1 between (what the compiler inserts in K2)
KERNEL(k_pair_nop1, "v_sub_co_u32 v48, vcc, v41, v42\n\ts_nop 1\n\tv_cndmask_b32 v49, v48, v41, vcc\n\t"
                    "v_sub_co_u32 v50, vcc, v42, v41\n\ts_nop 1\n\tv_cndmask_b32 v51, v50, v42, vcc\n\t")
// two consumers of one VCC
KERNEL(k_pair_two, "v_sub_co_u32 v48, vcc, v41, v42\n\tv_cndmask_b32 v49, v48, v41, vcc\n\tv_cndmask_b32 v50, v42, v41, vcc\n\t"
                   "v_sub_co_u32 v51, vcc, v42, v41\n\tv_cndmask_b32 v52, v51, v42, vcc\n\tv_cndmask_b32 v53, v41, v42, vcc\n\t")
// SGPR-pair carry (VOP3 forms)
KERNEL(k_pair_sgpr, "v_sub_co_u32_e64 v48, s[20:21], v41, v42\n\tv_cndmask_b32_e64 v49, v48, v41, s[20:21]\n\t"
                    "v_sub_co_u32_e64 v50, s[20:21], v42, v41\n\tv_cndmask_b32_e64 v51, v50, v42, s[20:21]\n\t")
// producer only (sub_co stream) and consumer of a stale VCC only
KERNEL(k_subco, "v_sub_co_u32 v48, vcc, v41, v42\n\tv_sub_co_u32 v49, vcc, v42, v41\n\t"
                "v_sub_co_u32 v50, vcc, v41, v43\n\tv_sub_co_u32 v51, vcc, v43, v41\n\t")
KERNEL(k_cnd_stale, "v_cndmask_b32 v48, v41, v42, vcc\n\tv_cndmask_b32 v49, v42, v41, vcc\n\t"
                    "v_cndmask_b32 v50, v41, v43, vcc\n\tv_cndmask_b32 v51, v43, v41, vcc\n\t")
// v_addc with VCC carry-in right after its producer (a 64-bit add in VOP2 form); below, the same with
// n independent VOP2 between (per pattern: 2 + n instructions)
KERNEL(k_addc_pair, "v_add_co_u32 v48, vcc, v41, v42\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t"
                    "v_add_co_u32 v50, vcc, v42, v41\n\tv_addc_co_u32 v51, vcc, v44, v43, vcc\n\t")

KERNEL(k_addc_gap0, "v_add_co_u32 v48, vcc, v41, v42\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t")
KERNEL(k_addc_gap2, "v_add_co_u32 v48, vcc, v41, v42\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t")
KERNEL(k_addc_gap4, "v_add_co_u32 v48, vcc, v41, v42\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t")
KERNEL(k_addc_gap8, "v_add_co_u32 v48, vcc, v41, v42\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t")
KERNEL(k_addc_gap12, "v_add_co_u32 v48, vcc, v41, v42\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_add_u32 v52, v43, v44\n\tv_add_u32 v53, v43, v44\n\tv_add_u32 v54, v43, v44\n\tv_add_u32 v55, v43, v44\n\tv_addc_co_u32 v49, vcc, v43, v44, vcc\n\t")

struct K {
    const char *n;
    void (*f)(uint32_t *, uint32_t);
};
static const K ks[] = {{"pair adjacent", k_pair_adj}, {"pair, 1 VOP2 between", k_pair_gap1},
                       {"pair, s_nop 1 between", k_pair_nop1}, {"pair + 2nd consumer", k_pair_two},
                       {"pair, SGPR carry (VOP3)", k_pair_sgpr}, {"sub_co only", k_subco},
                       {"cndmask stale VCC", k_cnd_stale}, {"add_co/addc pair", k_addc_pair},
                       {"add_co, 0 VOP2, addc", k_addc_gap0}, {"add_co, 2 VOP2, addc", k_addc_gap2}, {"add_co, 4 VOP2, addc", k_addc_gap4}, {"add_co, 8 VOP2, addc", k_addc_gap8}, {"add_co, 12 VOP2, addc", k_addc_gap12}};

int main() {
    const int cus = 256, blocks = cus * 8;  // 8 waves per SIMD
    uint32_t *out;
    (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
    hipEvent_t a, b;
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    for (const K &k : ks) {
        hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 7u);
        (void)hipDeviceSynchronize();
        (void)hipEventRecord(a);
        for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k.f, dim3(blocks), dim3(256), 0, 0, out, 7u);
        (void)hipEventRecord(b);
        (void)hipEventSynchronize(b);
        float ms;
        (void)hipEventElapsedTime(&ms, a, b);
        ms /= 3;
        // per 8-repeat block of one pattern: each KERNEL pattern above issues a fixed number of VALU
        // instructions; report time per pattern repeat (8 per asm block) per wave per SIMD
        const double reps = (double)blocks * 4 * ITERS * 8;  // pattern repeats (wave level)
        const double cyc = ms * 1e-3 * 2.4e9 / (reps / (cus * 4.0));
        printf("%-26s %8.3f ms %7.2f cyc/pattern/SIMD@2.4GHz\n", k.n, ms, cyc);
    }
    return 0;
}
