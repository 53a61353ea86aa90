#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
__global__ __launch_bounds__(256) void k0(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[0] = t1 - t0;
}
__global__ __launch_bounds__(256) void k1(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[1] = t1 - t0;
}
__global__ __launch_bounds__(256) void k2(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[2] = t1 - t0;
}
__global__ __launch_bounds__(256) void k3(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[3] = t1 - t0;
}
__global__ __launch_bounds__(256) void k4(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[4] = t1 - t0;
}
__global__ __launch_bounds__(256) void k5(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[5] = t1 - t0;
}
__global__ __launch_bounds__(256) void k6(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[6] = t1 - t0;
}
__global__ __launch_bounds__(256) void k7(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[7] = t1 - t0;
}
__global__ __launch_bounds__(256) void k8(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[8] = t1 - t0;
}
__global__ __launch_bounds__(256) void k9(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[9] = t1 - t0;
}
__global__ __launch_bounds__(256) void k10(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[10] = t1 - t0;
}
__global__ __launch_bounds__(256) void k11(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[11] = t1 - t0;
}
int main() {
  const int blocks = 256 * 8;  // 8 waves per SIMD
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1); float ms[64];
  uint32_t* out; uint64_t* clk; hipMalloc(&out, blocks * 256 * 4); hipMallocManaged(&clk, 64 * 8);
  hipLaunchKernelGGL(k0, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k0, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[0], e0, e1);
  hipLaunchKernelGGL(k1, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k1, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[1], e0, e1);
  hipLaunchKernelGGL(k2, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k2, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[2], e0, e1);
  hipLaunchKernelGGL(k3, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k3, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[3], e0, e1);
  hipLaunchKernelGGL(k4, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k4, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[4], e0, e1);
  hipLaunchKernelGGL(k5, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k5, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[5], e0, e1);
  hipLaunchKernelGGL(k6, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k6, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[6], e0, e1);
  hipLaunchKernelGGL(k7, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k7, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[7], e0, e1);
  hipLaunchKernelGGL(k8, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k8, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[8], e0, e1);
  hipLaunchKernelGGL(k9, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k9, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[9], e0, e1);
  hipLaunchKernelGGL(k10, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k10, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[10], e0, e1);
  hipLaunchKernelGGL(k11, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k11, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[11], e0, e1);
  const char* names[] = {"bitop3_vvv", "alignbit_vvv", "alignbit_vvs", "alignbit_vvi", "add_co", "addc_co", "bcnt", "and_or", "or_vv", "lshrrev_vs", "add_vs", "lshl_add_u64"};
  for (int n = 0; n < 12; ++n)
    printf("%-14s %.3f ms  %.2f cyc@2.4GHz per wave-instr per SIMD  (clock64 %.2f)\n", names[n], ms[n], ms[n] * 1e-3 * 2.4e9 / (4096 * 32.0 * 8.0), (double)clk[n] / (4096 * 32.0));
  return 0;
}
