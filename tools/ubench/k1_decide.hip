// Issue cost of the K1 decision sequences on gfx950 (cycles per wave-decision per SIMD at 2.4 GHz).
//   maxf64   : v_max_f64 alone (8 independent accumulators)
//   dec_f64  : decide_f64 (6 VOP2 + v_max_f64), 8 independent seeds
//   dec_u64  : decide_pos (10 VOP2), 8 independent seeds
// build: hipcc --offload-arch=gfx950 -O3 -o k1_decide k1_decide.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

#define ITERS 4096

#define F64_1(K, X)                                                                          \
    "v_sub_co_u32 %[t0], vcc, %[Tt], %[d]\n\t"                                                \
    "v_cndmask_b32 %[tmp], %[h2], %[h], vcc\n\t"                                              \
    "v_add_u32 " X ", " X ", %[tmp]\n\t"                                                      \
    "v_sub_co_u32 %[cv], vcc, " X ", %[mv]\n\t"                                               \
    "v_cndmask_b32 " X ", %[cv], " X ", vcc\n\t"                                              \
    "v_add_u32 %[part], %[part], " X "\n\t"                                                   \
    "v_max_f64 " K ", " K ", %[q]\n\t"

__global__ __launch_bounds__(256) void k_maxf64(uint32_t *out, uint32_t seed) {
    double a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
           a7 = seed + 7, q = threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
        asm volatile(
            "v_max_f64 %0, %0, %8\n\tv_max_f64 %1, %1, %8\n\tv_max_f64 %2, %2, %8\n\tv_max_f64 %3, %3, %8\n\t"
            "v_max_f64 %4, %4, %8\n\tv_max_f64 %5, %5, %8\n\tv_max_f64 %6, %6, %8\n\tv_max_f64 %7, %7, %8"
            : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3), "+v"(a4), "+v"(a5), "+v"(a6), "+v"(a7)
            : "v"(q));
    }
    out[blockIdx.x * 256 + threadIdx.x] = (uint32_t)(a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7);
}

__global__ __launch_bounds__(256) void k_dec_f64(uint32_t *out, uint32_t seed) {
    uint32_t t0, tmp, cv, part = 0, x0 = seed, x1 = seed + 1, x2 = seed + 2, x3 = seed + 3, x4 = seed + 4,
             x5 = seed + 5, x6 = seed + 6, x7 = seed + 7;
    uint32_t Tt = threadIdx.x, d = seed * 3, h = seed ^ 5, h2 = seed ^ 9, mv = 100000000;
    double k0 = 0, k1 = 0, k2 = 0, k3 = 0, k4 = 0, k5 = 0, k6 = 0, k7 = 0;
    double q = (double)threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
        asm volatile(F64_1("%[k0]", "%[x0]") F64_1("%[k1]", "%[x1]") F64_1("%[k2]", "%[x2]") F64_1("%[k3]", "%[x3]")
                         F64_1("%[k4]", "%[x4]") F64_1("%[k5]", "%[x5]") F64_1("%[k6]", "%[x6]") F64_1("%[k7]", "%[x7]")
                     : [t0] "=&v"(t0), [tmp] "=&v"(tmp), [cv] "=&v"(cv), [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2), [x3] "+v"(x3),
                       [x4] "+v"(x4), [x5] "+v"(x5), [x6] "+v"(x6), [x7] "+v"(x7), [part] "+v"(part),
                       [k0] "+v"(k0), [k1] "+v"(k1), [k2] "+v"(k2), [k3] "+v"(k3), [k4] "+v"(k4), [k5] "+v"(k5),
                       [k6] "+v"(k6), [k7] "+v"(k7)
                     : [Tt] "v"(Tt), [d] "v"(d), [h] "v"(h), [h2] "v"(h2), [mv] "v"(mv), [q] "v"(q)
                     : "vcc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = part + x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7 + (uint32_t)(k0 + k1 + k2 + k3 + k4 + k5 + k6 + k7);
}

#define U64_1                                            \
    "v_sub_co_u32 %[t0], vcc, %[Tt], %[d]\n\t"           \
    "v_cndmask_b32 %[sv], %[h2], %[h], vcc\n\t"          \
    "v_add_u32 %[sv], %[cm], %[sv]\n\t"                  \
    "v_sub_co_u32 %[cv], vcc, %[sv], %[mv]\n\t"          \
    "v_cndmask_b32 %[sv], %[cv], %[sv], vcc\n\t"         \
    "v_sub_co_u32 %[t0], vcc, %[klo], %[ne]\n\t"         \
    "v_subb_co_u32 %[t1], vcc, %[khi], %[sv], vcc\n\t"   \
    "v_cndmask_b32 %[klo], %[klo], %[ne], vcc\n\t"       \
    "v_cndmask_b32 %[khi], %[khi], %[sv], vcc\n\t"       \
    "v_add_u32 %[part], %[part], %[sv]\n\t"

__global__ __launch_bounds__(256) void k_dec_u64(uint32_t *out, uint32_t seed) {
    uint32_t t0, t1, sv, cv, part = 0, klo = 0, khi = 0;
    uint32_t Tt = threadIdx.x, d = seed * 3, h = seed ^ 5, h2 = seed ^ 9, mv = 100000000, cm = seed + 11,
             ne = ~threadIdx.x;
    for (int it = 0; it < ITERS; ++it) {
        asm volatile(U64_1 U64_1 U64_1 U64_1 U64_1 U64_1 U64_1 U64_1
                     : [t0] "=&v"(t0), [t1] "=&v"(t1), [sv] "=&v"(sv), [cv] "=&v"(cv), [klo] "+v"(klo),
                       [khi] "+v"(khi), [part] "+v"(part)
                     : [Tt] "v"(Tt), [d] "v"(d), [h] "v"(h), [h2] "v"(h2), [mv] "v"(mv), [cm] "v"(cm), [ne] "v"(ne)
                     : "vcc");
    }
    out[blockIdx.x * 256 + threadIdx.x] = part + klo + khi;
}

int main() {
    hipDeviceProp_t prop;
    (void)hipGetDeviceProperties(&prop, 0);
    const int cus = prop.multiProcessorCount;
    for (int wps = 2; wps <= 8; wps *= 2) {
        const int blocks = cus * wps;  // 4 waves per block = wps waves per SIMD
        uint32_t *out;
        (void)hipMalloc(&out, (size_t)blocks * 256 * 4);
        void (*ks[3])(uint32_t *, uint32_t) = {k_maxf64, k_dec_f64, k_dec_u64};
        const char *names[3] = {"maxf64 (1 instr)", "dec_f64 (7 instr)", "dec_u64 (10 instr)"};
        for (int i = 0; i < 3; ++i) {
            hipLaunchKernelGGL(ks[i], dim3(blocks), dim3(256), 0, 0, out, 1u);
            (void)hipDeviceSynchronize();
            hipEvent_t a, b;
            (void)hipEventCreate(&a);
            (void)hipEventCreate(&b);
            (void)hipEventRecord(a);
            hipLaunchKernelGGL(ks[i], dim3(blocks), dim3(256), 0, 0, out, 2u);
            (void)hipEventRecord(b);
            (void)hipEventSynchronize(b);
            float ms;
            (void)hipEventElapsedTime(&ms, a, b);
            const double per_simd = (double)ITERS * 8 * wps;  // wave-units (decisions or max) per SIMD
            printf("waves/SIMD=%d %-20s %8.3f ms  %6.2f cyc/wave-unit @2.4GHz\n", wps, names[i], ms,
                   ms * 1e-3 * 2.4e9 / per_simd);
        }
        (void)hipFree(out);
    }
    return 0;
}
