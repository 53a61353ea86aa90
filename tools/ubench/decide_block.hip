// Register-only throughput of K1's per-decision instruction block (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 2048

__device__ __forceinline__ void block_vcc(uint32_t Hlo, uint32_t Hhi, uint32_t Hm, uint32_t Hm2, uint32_t Clo,
                                          uint32_t Chi, uint32_t Cm, uint32_t ne, uint32_t mv, uint32_t &klo,
                                          uint32_t &khi, uint32_t &part) {
    uint32_t t0, t1, sv, cv;
    asm volatile("v_add_co_u32 %[t0], vcc, %[Clo], %[Hlo]\n\t"
        "v_addc_co_u32 %[t1], vcc, %[Chi], %[Hhi], vcc\n\t"
        "v_cndmask_b32 %[sv], %[Hm], %[Hm2], vcc\n\t"
        "v_add_u32 %[sv], %[Cm], %[sv]\n\t"
        "v_sub_co_u32 %[cv], vcc, %[sv], %[mv]\n\t"
        "v_cndmask_b32 %[sv], %[cv], %[sv], vcc\n\t"
        "v_sub_co_u32 %[t0], vcc, %[klo], %[ne]\n\t"
        "v_subb_co_u32 %[t1], vcc, %[khi], %[sv], vcc\n\t"
        "v_cndmask_b32 %[klo], %[klo], %[ne], vcc\n\t"
        "v_cndmask_b32 %[khi], %[khi], %[sv], vcc\n\t"
        "v_add_u32 %[part], %[part], %[sv]"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [sv] "=&v"(sv), [cv] "=&v"(cv), [klo] "+v"(klo), [khi] "+v"(khi),
          [part] "+v"(part)
        : [Hlo] "v"(Hlo), [Hhi] "v"(Hhi), [Hm] "v"(Hm), [Hm2] "v"(Hm2), [Clo] "v"(Clo), [Chi] "v"(Chi),
          [Cm] "v"(Cm), [ne] "v"(ne), [mv] "v"(mv) : "vcc");
}

template <int U, int NEV>
__global__ __launch_bounds__(256) void k(uint32_t* out, uint32_t seed) {
  uint32_t Hlo[U], Hhi[U], Hm[U], Hm2[U], klo[U], khi[U], part[U];
  for (int r = 0; r < U; ++r) { Hlo[r] = threadIdx.x * 3 + r; Hhi[r] = seed + r; Hm[r] = r; Hm2[r] = r + 1; klo[r] = 0; khi[r] = 0; part[r] = 0; }
  uint32_t C[NEV][4];
  for (int t = 0; t < NEV; ++t) { C[t][0] = seed * (t + 1); C[t][1] = seed ^ t; C[t][2] = t * 7; C[t][3] = ~t; }
  uint32_t mv = 100000000u + seed;
  for (int it = 0; it < ITERS; ++it) {
#pragma unroll
    for (int r = 0; r < U; ++r)
#pragma unroll
      for (int t = 0; t < NEV; ++t) {
        block_vcc(Hlo[r], Hhi[r], Hm[r], Hm2[r], C[t][0], C[t][1], C[t][2], C[t][3], mv, klo[r], khi[r], part[r]);
      }
  }
  uint32_t x = 0;
  for (int r = 0; r < U; ++r) x ^= klo[r] ^ khi[r] ^ part[r];
  out[blockIdx.x * 256 + threadIdx.x] = x;
}

template <int U, int NEV>
void run(const char* name, uint32_t* out, int waves_per_simd) {
  int blocks = 256 * waves_per_simd;  // 4 waves per block -> waves_per_simd per SIMD
  hipLaunchKernelGGL((k<U, NEV>), dim3(blocks), dim3(256), 0, 0, out, 7u);
  (void)hipDeviceSynchronize();
  hipEvent_t a, b; (void)hipEventCreate(&a); (void)hipEventCreate(&b);
  (void)hipEventRecord(a);
  for (int r = 0; r < 3; ++r) hipLaunchKernelGGL((k<U, NEV>), dim3(blocks), dim3(256), 0, 0, out, 7u);
  (void)hipEventRecord(b); (void)hipEventSynchronize(b);
  float ms; (void)hipEventElapsedTime(&ms, a, b); ms /= 3;
  double dec_per_simd = (double)waves_per_simd * ITERS * U * NEV;  // wave-decisions per SIMD
  double cyc = ms * 1e-3 * 2.4e9 / dec_per_simd;
  printf("%-28s waves/SIMD=%d  %7.3f ms  %6.2f cyc/wave-decision  (%.2f cyc/instr @11)\n", name, waves_per_simd, ms, cyc, cyc / 11);
}

int main() {
  uint32_t* out; (void)hipMalloc(&out, 256 * 16 * 256 * 4);
  for (int w : {1, 2, 4, 8}) run<2, 4>("U=2 NEV=4", out, w);
  for (int w : {2, 4, 6}) run<4, 4>("U=4 NEV=4", out, w);
  return 0;
}
