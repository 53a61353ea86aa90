// VGPR bank microbenchmark (gfx950): does a VOP2 whose two VGPR sources sit in the same bank
// (register index mod 4) issue slower than one whose sources sit in different banks?
// Question behind it: K1's decision sequence ends in v_cndmask_b32 x, cv, x with x and cv both
// allocated to registers = 3 (mod 4) for one seed of each lane.
// Build: hipcc --offload-arch=gfx950 -O3 -o vgpr_banks vgpr_banks.hip ; run on the box.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 8192
#define R8(X) X X X X X X X X
#define CLOB "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55"

// 32 independent instructions per asm block: destinations rotate over v48..v55
#define BODY(OP, A, B)                                                                                   \
    R8(OP " v48, " A ", " B "\n\t" OP " v49, " A ", " B "\n\t" OP " v50, " A ", " B "\n\t" OP " v51, " A \
       ", " B "\n\t")

#define KERNEL(NAME, OP, A, B)                                                                      \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                    \
        asm volatile("v_mov_b32 v40, %0\n\tv_mov_b32 v41, %0\n\tv_mov_b32 v44, %0\n\tv_mov_b32 v45, %0\n\t" \
                     "v_mov_b32 v42, %0\n\tv_mov_b32 v46, %0" ::"v"(seed + threadIdx.x)                   \
                     : CLOB);                                                                         \
        for (int it = 0; it < ITERS; ++it) asm volatile(BODY(OP, A, B)::: CLOB, "vcc");             \
        uint32_t r;                                                                                   \
        asm volatile("v_xor_b32 %0, v48, v51" : "=v"(r)::CLOB);                                        \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                                     \
    }

KERNEL(k_add_same, "v_add_u32", "v40", "v44")         // banks 0, 0
KERNEL(k_add_diff, "v_add_u32", "v40", "v41")         // banks 0, 1
KERNEL(k_xor_same, "v_xor_b32", "v41", "v45")         // banks 1, 1
KERNEL(k_xor_diff, "v_xor_b32", "v41", "v42")         // banks 1, 2

// v_cndmask with an explicit VCC operand
#define BODYC(A, B)                                                                                        \
    R8("v_cndmask_b32 v48, " A ", " B ", vcc\n\tv_cndmask_b32 v49, " A ", " B ", vcc\n\t"                 \
       "v_cndmask_b32 v50, " A ", " B ", vcc\n\tv_cndmask_b32 v51, " A ", " B ", vcc\n\t")
#define KERNELC(NAME, A, B)                                                                         \
    __global__ __launch_bounds__(256) void NAME(uint32_t *out, uint32_t seed) {                    \
        asm volatile("v_mov_b32 v40, %0\n\tv_mov_b32 v41, %0\n\tv_mov_b32 v44, %0\n\tv_mov_b32 v45, %0\n\t" \
                     "v_mov_b32 v42, %0\n\tv_mov_b32 v46, %0\n\tv_cmp_gt_u32 vcc, 17, %0" ::"v"(seed + threadIdx.x) \
                     : CLOB, "vcc");                                                                  \
        for (int it = 0; it < ITERS; ++it) asm volatile(BODYC(A, B)::: CLOB, "vcc");               \
        uint32_t r;                                                                                   \
        asm volatile("v_xor_b32 %0, v48, v51" : "=v"(r)::CLOB);                                        \
        out[blockIdx.x * 256 + threadIdx.x] = r;                                                     \
    }
KERNELC(k_cndm_same, "v41", "v45")  // banks 1, 1
KERNELC(k_cndm_diff, "v41", "v42")  // banks 1, 2

struct K {
    const char *n;
    void (*f)(uint32_t *, uint32_t);
};
static const K ks[] = {{"add same bank", k_add_same}, {"add diff bank", k_add_diff},
                       {"xor same bank", k_xor_same}, {"xor diff bank", k_xor_diff},
                       {"cndmask same bank", k_cndm_same}, {"cndmask diff bank", k_cndm_diff},
                       {"add same bank (rep)", k_add_same}, {"add diff bank (rep)", k_add_diff}};

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
        const double wi = (double)blocks * 4 * ITERS * 32;  // wave-instructions
        const double cyc = ms * 1e-3 * 2.4e9 / (wi / (cus * 4.0));
        printf("%-22s %8.3f ms %6.2f cyc/wave-instr/SIMD@2.4GHz\n", k.n, ms, cyc);
    }
    return 0;
}
