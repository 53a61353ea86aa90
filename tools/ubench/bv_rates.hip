#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#define ITERS 4096
__global__ __launch_bounds__(256) void k0(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], %[b] bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], %[b] bitop3:0xf1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]\n\tv_alignbit_b32 %0, %0, %[a], %[b]\n\tv_alignbit_b32 %1, %1, %[a], %[b]\n\tv_alignbit_b32 %2, %2, %[a], %[b]\n\tv_alignbit_b32 %3, %3, %[a], %[b]\n\tv_alignbit_b32 %4, %4, %[a], %[b]\n\tv_alignbit_b32 %5, %5, %[a], %[b]\n\tv_alignbit_b32 %6, %6, %[a], %[b]\n\tv_alignbit_b32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]\n\tv_alignbit_b32 %0, %0, %[a], %[sg]\n\tv_alignbit_b32 %1, %1, %[a], %[sg]\n\tv_alignbit_b32 %2, %2, %[a], %[sg]\n\tv_alignbit_b32 %3, %3, %[a], %[sg]\n\tv_alignbit_b32 %4, %4, %[a], %[sg]\n\tv_alignbit_b32 %5, %5, %[a], %[sg]\n\tv_alignbit_b32 %6, %6, %[a], %[sg]\n\tv_alignbit_b32 %7, %7, %[a], %[sg]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1\n\tv_alignbit_b32 %0, %0, %[a], 1\n\tv_alignbit_b32 %1, %1, %[a], 1\n\tv_alignbit_b32 %2, %2, %[a], 1\n\tv_alignbit_b32 %3, %3, %[a], 1\n\tv_alignbit_b32 %4, %4, %[a], 1\n\tv_alignbit_b32 %5, %5, %[a], 1\n\tv_alignbit_b32 %6, %6, %[a], 1\n\tv_alignbit_b32 %7, %7, %[a], 1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]\n\tv_add_co_u32 %0, vcc, %0, %[a]\n\tv_add_co_u32 %1, vcc, %1, %[a]\n\tv_add_co_u32 %2, vcc, %2, %[a]\n\tv_add_co_u32 %3, vcc, %3, %[a]\n\tv_add_co_u32 %4, vcc, %4, %[a]\n\tv_add_co_u32 %5, vcc, %5, %[a]\n\tv_add_co_u32 %6, vcc, %6, %[a]\n\tv_add_co_u32 %7, vcc, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc\n\tv_addc_co_u32 %0, vcc, %0, %[a], vcc\n\tv_addc_co_u32 %1, vcc, %1, %[a], vcc\n\tv_addc_co_u32 %2, vcc, %2, %[a], vcc\n\tv_addc_co_u32 %3, vcc, %3, %[a], vcc\n\tv_addc_co_u32 %4, vcc, %4, %[a], vcc\n\tv_addc_co_u32 %5, vcc, %5, %[a], vcc\n\tv_addc_co_u32 %6, vcc, %6, %[a], vcc\n\tv_addc_co_u32 %7, vcc, %7, %[a], vcc" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]\n\tv_bcnt_u32_b32 %0, %0, %[a]\n\tv_bcnt_u32_b32 %1, %1, %[a]\n\tv_bcnt_u32_b32 %2, %2, %[a]\n\tv_bcnt_u32_b32 %3, %3, %[a]\n\tv_bcnt_u32_b32 %4, %4, %[a]\n\tv_bcnt_u32_b32 %5, %5, %[a]\n\tv_bcnt_u32_b32 %6, %6, %[a]\n\tv_bcnt_u32_b32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]\n\tv_and_or_b32 %0, %0, %[a], %[b]\n\tv_and_or_b32 %1, %1, %[a], %[b]\n\tv_and_or_b32 %2, %2, %[a], %[b]\n\tv_and_or_b32 %3, %3, %[a], %[b]\n\tv_and_or_b32 %4, %4, %[a], %[b]\n\tv_and_or_b32 %5, %5, %[a], %[b]\n\tv_and_or_b32 %6, %6, %[a], %[b]\n\tv_and_or_b32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]\n\tv_or_b32 %0, %0, %[a]\n\tv_or_b32 %1, %1, %[a]\n\tv_or_b32 %2, %2, %[a]\n\tv_or_b32 %3, %3, %[a]\n\tv_or_b32 %4, %4, %[a]\n\tv_or_b32 %5, %5, %[a]\n\tv_or_b32 %6, %6, %[a]\n\tv_or_b32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7\n\tv_lshrrev_b32 %0, %[sg], %0\n\tv_lshrrev_b32 %1, %[sg], %1\n\tv_lshrrev_b32 %2, %[sg], %2\n\tv_lshrrev_b32 %3, %[sg], %3\n\tv_lshrrev_b32 %4, %[sg], %4\n\tv_lshrrev_b32 %5, %[sg], %5\n\tv_lshrrev_b32 %6, %[sg], %6\n\tv_lshrrev_b32 %7, %[sg], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7\n\tv_add_u32 %0, %[sg], %0\n\tv_add_u32 %1, %[sg], %1\n\tv_add_u32 %2, %[sg], %2\n\tv_add_u32 %3, %[sg], %3\n\tv_add_u32 %4, %[sg], %4\n\tv_add_u32 %5, %[sg], %5\n\tv_add_u32 %6, %[sg], %6\n\tv_add_u32 %7, %[sg], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
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
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]\n\tv_lshl_add_u64 %[w0], %[w0], 0, %[wa]\n\tv_lshl_add_u64 %[w1], %[w1], 0, %[wa]\n\tv_lshl_add_u64 %[w2], %[w2], 0, %[wa]\n\tv_lshl_add_u64 %[w3], %[w3], 0, %[wa]\n\tv_lshl_add_u64 %[w4], %[w4], 0, %[wa]\n\tv_lshl_add_u64 %[w5], %[w5], 0, %[wa]\n\tv_lshl_add_u64 %[w6], %[w6], 0, %[wa]\n\tv_lshl_add_u64 %[w7], %[w7], 0, %[wa]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[11] = t1 - t0;
}
__global__ __launch_bounds__(256) void k12(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshrrev_b32 %0, %[a], %0\n\tv_lshrrev_b32 %1, %[a], %1\n\tv_lshrrev_b32 %2, %[a], %2\n\tv_lshrrev_b32 %3, %[a], %3\n\tv_lshrrev_b32 %4, %[a], %4\n\tv_lshrrev_b32 %5, %[a], %5\n\tv_lshrrev_b32 %6, %[a], %6\n\tv_lshrrev_b32 %7, %[a], %7\n\tv_lshrrev_b32 %0, %[a], %0\n\tv_lshrrev_b32 %1, %[a], %1\n\tv_lshrrev_b32 %2, %[a], %2\n\tv_lshrrev_b32 %3, %[a], %3\n\tv_lshrrev_b32 %4, %[a], %4\n\tv_lshrrev_b32 %5, %[a], %5\n\tv_lshrrev_b32 %6, %[a], %6\n\tv_lshrrev_b32 %7, %[a], %7\n\tv_lshrrev_b32 %0, %[a], %0\n\tv_lshrrev_b32 %1, %[a], %1\n\tv_lshrrev_b32 %2, %[a], %2\n\tv_lshrrev_b32 %3, %[a], %3\n\tv_lshrrev_b32 %4, %[a], %4\n\tv_lshrrev_b32 %5, %[a], %5\n\tv_lshrrev_b32 %6, %[a], %6\n\tv_lshrrev_b32 %7, %[a], %7\n\tv_lshrrev_b32 %0, %[a], %0\n\tv_lshrrev_b32 %1, %[a], %1\n\tv_lshrrev_b32 %2, %[a], %2\n\tv_lshrrev_b32 %3, %[a], %3\n\tv_lshrrev_b32 %4, %[a], %4\n\tv_lshrrev_b32 %5, %[a], %5\n\tv_lshrrev_b32 %6, %[a], %6\n\tv_lshrrev_b32 %7, %[a], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[12] = t1 - t0;
}
__global__ __launch_bounds__(256) void k13(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 3, %1\n\tv_lshrrev_b32 %2, 3, %2\n\tv_lshrrev_b32 %3, 3, %3\n\tv_lshrrev_b32 %4, 3, %4\n\tv_lshrrev_b32 %5, 3, %5\n\tv_lshrrev_b32 %6, 3, %6\n\tv_lshrrev_b32 %7, 3, %7\n\tv_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 3, %1\n\tv_lshrrev_b32 %2, 3, %2\n\tv_lshrrev_b32 %3, 3, %3\n\tv_lshrrev_b32 %4, 3, %4\n\tv_lshrrev_b32 %5, 3, %5\n\tv_lshrrev_b32 %6, 3, %6\n\tv_lshrrev_b32 %7, 3, %7\n\tv_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 3, %1\n\tv_lshrrev_b32 %2, 3, %2\n\tv_lshrrev_b32 %3, 3, %3\n\tv_lshrrev_b32 %4, 3, %4\n\tv_lshrrev_b32 %5, 3, %5\n\tv_lshrrev_b32 %6, 3, %6\n\tv_lshrrev_b32 %7, 3, %7\n\tv_lshrrev_b32 %0, 3, %0\n\tv_lshrrev_b32 %1, 3, %1\n\tv_lshrrev_b32 %2, 3, %2\n\tv_lshrrev_b32 %3, 3, %3\n\tv_lshrrev_b32 %4, 3, %4\n\tv_lshrrev_b32 %5, 3, %5\n\tv_lshrrev_b32 %6, 3, %6\n\tv_lshrrev_b32 %7, 3, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[13] = t1 - t0;
}
__global__ __launch_bounds__(256) void k14(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_xor_b32 %0, 1, %0\n\tv_xor_b32 %1, 1, %1\n\tv_xor_b32 %2, 1, %2\n\tv_xor_b32 %3, 1, %3\n\tv_xor_b32 %4, 1, %4\n\tv_xor_b32 %5, 1, %5\n\tv_xor_b32 %6, 1, %6\n\tv_xor_b32 %7, 1, %7\n\tv_xor_b32 %0, 1, %0\n\tv_xor_b32 %1, 1, %1\n\tv_xor_b32 %2, 1, %2\n\tv_xor_b32 %3, 1, %3\n\tv_xor_b32 %4, 1, %4\n\tv_xor_b32 %5, 1, %5\n\tv_xor_b32 %6, 1, %6\n\tv_xor_b32 %7, 1, %7\n\tv_xor_b32 %0, 1, %0\n\tv_xor_b32 %1, 1, %1\n\tv_xor_b32 %2, 1, %2\n\tv_xor_b32 %3, 1, %3\n\tv_xor_b32 %4, 1, %4\n\tv_xor_b32 %5, 1, %5\n\tv_xor_b32 %6, 1, %6\n\tv_xor_b32 %7, 1, %7\n\tv_xor_b32 %0, 1, %0\n\tv_xor_b32 %1, 1, %1\n\tv_xor_b32 %2, 1, %2\n\tv_xor_b32 %3, 1, %3\n\tv_xor_b32 %4, 1, %4\n\tv_xor_b32 %5, 1, %5\n\tv_xor_b32 %6, 1, %6\n\tv_xor_b32 %7, 1, %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[14] = t1 - t0;
}
__global__ __launch_bounds__(256) void k15(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_xor_b32 %0, %[a], %0\n\tv_xor_b32 %1, %[a], %1\n\tv_xor_b32 %2, %[a], %2\n\tv_xor_b32 %3, %[a], %3\n\tv_xor_b32 %4, %[a], %4\n\tv_xor_b32 %5, %[a], %5\n\tv_xor_b32 %6, %[a], %6\n\tv_xor_b32 %7, %[a], %7\n\tv_xor_b32 %0, %[a], %0\n\tv_xor_b32 %1, %[a], %1\n\tv_xor_b32 %2, %[a], %2\n\tv_xor_b32 %3, %[a], %3\n\tv_xor_b32 %4, %[a], %4\n\tv_xor_b32 %5, %[a], %5\n\tv_xor_b32 %6, %[a], %6\n\tv_xor_b32 %7, %[a], %7\n\tv_xor_b32 %0, %[a], %0\n\tv_xor_b32 %1, %[a], %1\n\tv_xor_b32 %2, %[a], %2\n\tv_xor_b32 %3, %[a], %3\n\tv_xor_b32 %4, %[a], %4\n\tv_xor_b32 %5, %[a], %5\n\tv_xor_b32 %6, %[a], %6\n\tv_xor_b32 %7, %[a], %7\n\tv_xor_b32 %0, %[a], %0\n\tv_xor_b32 %1, %[a], %1\n\tv_xor_b32 %2, %[a], %2\n\tv_xor_b32 %3, %[a], %3\n\tv_xor_b32 %4, %[a], %4\n\tv_xor_b32 %5, %[a], %5\n\tv_xor_b32 %6, %[a], %6\n\tv_xor_b32 %7, %[a], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[15] = t1 - t0;
}
__global__ __launch_bounds__(256) void k16(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_add3_u32 %0, %0, %[a], %[b]\n\tv_add3_u32 %1, %1, %[a], %[b]\n\tv_add3_u32 %2, %2, %[a], %[b]\n\tv_add3_u32 %3, %3, %[a], %[b]\n\tv_add3_u32 %4, %4, %[a], %[b]\n\tv_add3_u32 %5, %5, %[a], %[b]\n\tv_add3_u32 %6, %6, %[a], %[b]\n\tv_add3_u32 %7, %7, %[a], %[b]\n\tv_add3_u32 %0, %0, %[a], %[b]\n\tv_add3_u32 %1, %1, %[a], %[b]\n\tv_add3_u32 %2, %2, %[a], %[b]\n\tv_add3_u32 %3, %3, %[a], %[b]\n\tv_add3_u32 %4, %4, %[a], %[b]\n\tv_add3_u32 %5, %5, %[a], %[b]\n\tv_add3_u32 %6, %6, %[a], %[b]\n\tv_add3_u32 %7, %7, %[a], %[b]\n\tv_add3_u32 %0, %0, %[a], %[b]\n\tv_add3_u32 %1, %1, %[a], %[b]\n\tv_add3_u32 %2, %2, %[a], %[b]\n\tv_add3_u32 %3, %3, %[a], %[b]\n\tv_add3_u32 %4, %4, %[a], %[b]\n\tv_add3_u32 %5, %5, %[a], %[b]\n\tv_add3_u32 %6, %6, %[a], %[b]\n\tv_add3_u32 %7, %7, %[a], %[b]\n\tv_add3_u32 %0, %0, %[a], %[b]\n\tv_add3_u32 %1, %1, %[a], %[b]\n\tv_add3_u32 %2, %2, %[a], %[b]\n\tv_add3_u32 %3, %3, %[a], %[b]\n\tv_add3_u32 %4, %4, %[a], %[b]\n\tv_add3_u32 %5, %5, %[a], %[b]\n\tv_add3_u32 %6, %6, %[a], %[b]\n\tv_add3_u32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[16] = t1 - t0;
}
__global__ __launch_bounds__(256) void k17(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_lshl_add_u32 %0, %0, 2, %[a]\n\tv_lshl_add_u32 %1, %1, 2, %[a]\n\tv_lshl_add_u32 %2, %2, 2, %[a]\n\tv_lshl_add_u32 %3, %3, 2, %[a]\n\tv_lshl_add_u32 %4, %4, 2, %[a]\n\tv_lshl_add_u32 %5, %5, 2, %[a]\n\tv_lshl_add_u32 %6, %6, 2, %[a]\n\tv_lshl_add_u32 %7, %7, 2, %[a]\n\tv_lshl_add_u32 %0, %0, 2, %[a]\n\tv_lshl_add_u32 %1, %1, 2, %[a]\n\tv_lshl_add_u32 %2, %2, 2, %[a]\n\tv_lshl_add_u32 %3, %3, 2, %[a]\n\tv_lshl_add_u32 %4, %4, 2, %[a]\n\tv_lshl_add_u32 %5, %5, 2, %[a]\n\tv_lshl_add_u32 %6, %6, 2, %[a]\n\tv_lshl_add_u32 %7, %7, 2, %[a]\n\tv_lshl_add_u32 %0, %0, 2, %[a]\n\tv_lshl_add_u32 %1, %1, 2, %[a]\n\tv_lshl_add_u32 %2, %2, 2, %[a]\n\tv_lshl_add_u32 %3, %3, 2, %[a]\n\tv_lshl_add_u32 %4, %4, 2, %[a]\n\tv_lshl_add_u32 %5, %5, 2, %[a]\n\tv_lshl_add_u32 %6, %6, 2, %[a]\n\tv_lshl_add_u32 %7, %7, 2, %[a]\n\tv_lshl_add_u32 %0, %0, 2, %[a]\n\tv_lshl_add_u32 %1, %1, 2, %[a]\n\tv_lshl_add_u32 %2, %2, 2, %[a]\n\tv_lshl_add_u32 %3, %3, 2, %[a]\n\tv_lshl_add_u32 %4, %4, 2, %[a]\n\tv_lshl_add_u32 %5, %5, 2, %[a]\n\tv_lshl_add_u32 %6, %6, 2, %[a]\n\tv_lshl_add_u32 %7, %7, 2, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[17] = t1 - t0;
}
__global__ __launch_bounds__(256) void k18(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bfe_u32 %0, %0, %[a], %[b]\n\tv_bfe_u32 %1, %1, %[a], %[b]\n\tv_bfe_u32 %2, %2, %[a], %[b]\n\tv_bfe_u32 %3, %3, %[a], %[b]\n\tv_bfe_u32 %4, %4, %[a], %[b]\n\tv_bfe_u32 %5, %5, %[a], %[b]\n\tv_bfe_u32 %6, %6, %[a], %[b]\n\tv_bfe_u32 %7, %7, %[a], %[b]\n\tv_bfe_u32 %0, %0, %[a], %[b]\n\tv_bfe_u32 %1, %1, %[a], %[b]\n\tv_bfe_u32 %2, %2, %[a], %[b]\n\tv_bfe_u32 %3, %3, %[a], %[b]\n\tv_bfe_u32 %4, %4, %[a], %[b]\n\tv_bfe_u32 %5, %5, %[a], %[b]\n\tv_bfe_u32 %6, %6, %[a], %[b]\n\tv_bfe_u32 %7, %7, %[a], %[b]\n\tv_bfe_u32 %0, %0, %[a], %[b]\n\tv_bfe_u32 %1, %1, %[a], %[b]\n\tv_bfe_u32 %2, %2, %[a], %[b]\n\tv_bfe_u32 %3, %3, %[a], %[b]\n\tv_bfe_u32 %4, %4, %[a], %[b]\n\tv_bfe_u32 %5, %5, %[a], %[b]\n\tv_bfe_u32 %6, %6, %[a], %[b]\n\tv_bfe_u32 %7, %7, %[a], %[b]\n\tv_bfe_u32 %0, %0, %[a], %[b]\n\tv_bfe_u32 %1, %1, %[a], %[b]\n\tv_bfe_u32 %2, %2, %[a], %[b]\n\tv_bfe_u32 %3, %3, %[a], %[b]\n\tv_bfe_u32 %4, %4, %[a], %[b]\n\tv_bfe_u32 %5, %5, %[a], %[b]\n\tv_bfe_u32 %6, %6, %[a], %[b]\n\tv_bfe_u32 %7, %7, %[a], %[b]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[18] = t1 - t0;
}
__global__ __launch_bounds__(256) void k19(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bcnt_u32_b32 %0, %0, 0\n\tv_bcnt_u32_b32 %1, %1, 0\n\tv_bcnt_u32_b32 %2, %2, 0\n\tv_bcnt_u32_b32 %3, %3, 0\n\tv_bcnt_u32_b32 %4, %4, 0\n\tv_bcnt_u32_b32 %5, %5, 0\n\tv_bcnt_u32_b32 %6, %6, 0\n\tv_bcnt_u32_b32 %7, %7, 0\n\tv_bcnt_u32_b32 %0, %0, 0\n\tv_bcnt_u32_b32 %1, %1, 0\n\tv_bcnt_u32_b32 %2, %2, 0\n\tv_bcnt_u32_b32 %3, %3, 0\n\tv_bcnt_u32_b32 %4, %4, 0\n\tv_bcnt_u32_b32 %5, %5, 0\n\tv_bcnt_u32_b32 %6, %6, 0\n\tv_bcnt_u32_b32 %7, %7, 0\n\tv_bcnt_u32_b32 %0, %0, 0\n\tv_bcnt_u32_b32 %1, %1, 0\n\tv_bcnt_u32_b32 %2, %2, 0\n\tv_bcnt_u32_b32 %3, %3, 0\n\tv_bcnt_u32_b32 %4, %4, 0\n\tv_bcnt_u32_b32 %5, %5, 0\n\tv_bcnt_u32_b32 %6, %6, 0\n\tv_bcnt_u32_b32 %7, %7, 0\n\tv_bcnt_u32_b32 %0, %0, 0\n\tv_bcnt_u32_b32 %1, %1, 0\n\tv_bcnt_u32_b32 %2, %2, 0\n\tv_bcnt_u32_b32 %3, %3, 0\n\tv_bcnt_u32_b32 %4, %4, 0\n\tv_bcnt_u32_b32 %5, %5, 0\n\tv_bcnt_u32_b32 %6, %6, 0\n\tv_bcnt_u32_b32 %7, %7, 0" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[19] = t1 - t0;
}
__global__ __launch_bounds__(256) void k20(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_cndmask_b32 %0, %0, %[a], vcc\n\tv_cndmask_b32 %1, %1, %[a], vcc\n\tv_cndmask_b32 %2, %2, %[a], vcc\n\tv_cndmask_b32 %3, %3, %[a], vcc\n\tv_cndmask_b32 %4, %4, %[a], vcc\n\tv_cndmask_b32 %5, %5, %[a], vcc\n\tv_cndmask_b32 %6, %6, %[a], vcc\n\tv_cndmask_b32 %7, %7, %[a], vcc\n\tv_cndmask_b32 %0, %0, %[a], vcc\n\tv_cndmask_b32 %1, %1, %[a], vcc\n\tv_cndmask_b32 %2, %2, %[a], vcc\n\tv_cndmask_b32 %3, %3, %[a], vcc\n\tv_cndmask_b32 %4, %4, %[a], vcc\n\tv_cndmask_b32 %5, %5, %[a], vcc\n\tv_cndmask_b32 %6, %6, %[a], vcc\n\tv_cndmask_b32 %7, %7, %[a], vcc\n\tv_cndmask_b32 %0, %0, %[a], vcc\n\tv_cndmask_b32 %1, %1, %[a], vcc\n\tv_cndmask_b32 %2, %2, %[a], vcc\n\tv_cndmask_b32 %3, %3, %[a], vcc\n\tv_cndmask_b32 %4, %4, %[a], vcc\n\tv_cndmask_b32 %5, %5, %[a], vcc\n\tv_cndmask_b32 %6, %6, %[a], vcc\n\tv_cndmask_b32 %7, %7, %[a], vcc\n\tv_cndmask_b32 %0, %0, %[a], vcc\n\tv_cndmask_b32 %1, %1, %[a], vcc\n\tv_cndmask_b32 %2, %2, %[a], vcc\n\tv_cndmask_b32 %3, %3, %[a], vcc\n\tv_cndmask_b32 %4, %4, %[a], vcc\n\tv_cndmask_b32 %5, %5, %[a], vcc\n\tv_cndmask_b32 %6, %6, %[a], vcc\n\tv_cndmask_b32 %7, %7, %[a], vcc" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[20] = t1 - t0;
}
__global__ __launch_bounds__(256) void k21(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_cndmask_b32_e64 %0, %0, %[a], %[sm]\n\tv_cndmask_b32_e64 %1, %1, %[a], %[sm]\n\tv_cndmask_b32_e64 %2, %2, %[a], %[sm]\n\tv_cndmask_b32_e64 %3, %3, %[a], %[sm]\n\tv_cndmask_b32_e64 %4, %4, %[a], %[sm]\n\tv_cndmask_b32_e64 %5, %5, %[a], %[sm]\n\tv_cndmask_b32_e64 %6, %6, %[a], %[sm]\n\tv_cndmask_b32_e64 %7, %7, %[a], %[sm]\n\tv_cndmask_b32_e64 %0, %0, %[a], %[sm]\n\tv_cndmask_b32_e64 %1, %1, %[a], %[sm]\n\tv_cndmask_b32_e64 %2, %2, %[a], %[sm]\n\tv_cndmask_b32_e64 %3, %3, %[a], %[sm]\n\tv_cndmask_b32_e64 %4, %4, %[a], %[sm]\n\tv_cndmask_b32_e64 %5, %5, %[a], %[sm]\n\tv_cndmask_b32_e64 %6, %6, %[a], %[sm]\n\tv_cndmask_b32_e64 %7, %7, %[a], %[sm]\n\tv_cndmask_b32_e64 %0, %0, %[a], %[sm]\n\tv_cndmask_b32_e64 %1, %1, %[a], %[sm]\n\tv_cndmask_b32_e64 %2, %2, %[a], %[sm]\n\tv_cndmask_b32_e64 %3, %3, %[a], %[sm]\n\tv_cndmask_b32_e64 %4, %4, %[a], %[sm]\n\tv_cndmask_b32_e64 %5, %5, %[a], %[sm]\n\tv_cndmask_b32_e64 %6, %6, %[a], %[sm]\n\tv_cndmask_b32_e64 %7, %7, %[a], %[sm]\n\tv_cndmask_b32_e64 %0, %0, %[a], %[sm]\n\tv_cndmask_b32_e64 %1, %1, %[a], %[sm]\n\tv_cndmask_b32_e64 %2, %2, %[a], %[sm]\n\tv_cndmask_b32_e64 %3, %3, %[a], %[sm]\n\tv_cndmask_b32_e64 %4, %4, %[a], %[sm]\n\tv_cndmask_b32_e64 %5, %5, %[a], %[sm]\n\tv_cndmask_b32_e64 %6, %6, %[a], %[sm]\n\tv_cndmask_b32_e64 %7, %7, %[a], %[sm]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[21] = t1 - t0;
}
__global__ __launch_bounds__(256) void k22(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_min_u32 %0, %0, %[a]\n\tv_min_u32 %1, %1, %[a]\n\tv_min_u32 %2, %2, %[a]\n\tv_min_u32 %3, %3, %[a]\n\tv_min_u32 %4, %4, %[a]\n\tv_min_u32 %5, %5, %[a]\n\tv_min_u32 %6, %6, %[a]\n\tv_min_u32 %7, %7, %[a]\n\tv_min_u32 %0, %0, %[a]\n\tv_min_u32 %1, %1, %[a]\n\tv_min_u32 %2, %2, %[a]\n\tv_min_u32 %3, %3, %[a]\n\tv_min_u32 %4, %4, %[a]\n\tv_min_u32 %5, %5, %[a]\n\tv_min_u32 %6, %6, %[a]\n\tv_min_u32 %7, %7, %[a]\n\tv_min_u32 %0, %0, %[a]\n\tv_min_u32 %1, %1, %[a]\n\tv_min_u32 %2, %2, %[a]\n\tv_min_u32 %3, %3, %[a]\n\tv_min_u32 %4, %4, %[a]\n\tv_min_u32 %5, %5, %[a]\n\tv_min_u32 %6, %6, %[a]\n\tv_min_u32 %7, %7, %[a]\n\tv_min_u32 %0, %0, %[a]\n\tv_min_u32 %1, %1, %[a]\n\tv_min_u32 %2, %2, %[a]\n\tv_min_u32 %3, %3, %[a]\n\tv_min_u32 %4, %4, %[a]\n\tv_min_u32 %5, %5, %[a]\n\tv_min_u32 %6, %6, %[a]\n\tv_min_u32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[22] = t1 - t0;
}
__global__ __launch_bounds__(256) void k23(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mul_hi_u32 %0, %0, %[a]\n\tv_mul_hi_u32 %1, %1, %[a]\n\tv_mul_hi_u32 %2, %2, %[a]\n\tv_mul_hi_u32 %3, %3, %[a]\n\tv_mul_hi_u32 %4, %4, %[a]\n\tv_mul_hi_u32 %5, %5, %[a]\n\tv_mul_hi_u32 %6, %6, %[a]\n\tv_mul_hi_u32 %7, %7, %[a]\n\tv_mul_hi_u32 %0, %0, %[a]\n\tv_mul_hi_u32 %1, %1, %[a]\n\tv_mul_hi_u32 %2, %2, %[a]\n\tv_mul_hi_u32 %3, %3, %[a]\n\tv_mul_hi_u32 %4, %4, %[a]\n\tv_mul_hi_u32 %5, %5, %[a]\n\tv_mul_hi_u32 %6, %6, %[a]\n\tv_mul_hi_u32 %7, %7, %[a]\n\tv_mul_hi_u32 %0, %0, %[a]\n\tv_mul_hi_u32 %1, %1, %[a]\n\tv_mul_hi_u32 %2, %2, %[a]\n\tv_mul_hi_u32 %3, %3, %[a]\n\tv_mul_hi_u32 %4, %4, %[a]\n\tv_mul_hi_u32 %5, %5, %[a]\n\tv_mul_hi_u32 %6, %6, %[a]\n\tv_mul_hi_u32 %7, %7, %[a]\n\tv_mul_hi_u32 %0, %0, %[a]\n\tv_mul_hi_u32 %1, %1, %[a]\n\tv_mul_hi_u32 %2, %2, %[a]\n\tv_mul_hi_u32 %3, %3, %[a]\n\tv_mul_hi_u32 %4, %4, %[a]\n\tv_mul_hi_u32 %5, %5, %[a]\n\tv_mul_hi_u32 %6, %6, %[a]\n\tv_mul_hi_u32 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[23] = t1 - t0;
}
__global__ __launch_bounds__(256) void k24(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mul_u32_u24 %0, %0, %[a]\n\tv_mul_u32_u24 %1, %1, %[a]\n\tv_mul_u32_u24 %2, %2, %[a]\n\tv_mul_u32_u24 %3, %3, %[a]\n\tv_mul_u32_u24 %4, %4, %[a]\n\tv_mul_u32_u24 %5, %5, %[a]\n\tv_mul_u32_u24 %6, %6, %[a]\n\tv_mul_u32_u24 %7, %7, %[a]\n\tv_mul_u32_u24 %0, %0, %[a]\n\tv_mul_u32_u24 %1, %1, %[a]\n\tv_mul_u32_u24 %2, %2, %[a]\n\tv_mul_u32_u24 %3, %3, %[a]\n\tv_mul_u32_u24 %4, %4, %[a]\n\tv_mul_u32_u24 %5, %5, %[a]\n\tv_mul_u32_u24 %6, %6, %[a]\n\tv_mul_u32_u24 %7, %7, %[a]\n\tv_mul_u32_u24 %0, %0, %[a]\n\tv_mul_u32_u24 %1, %1, %[a]\n\tv_mul_u32_u24 %2, %2, %[a]\n\tv_mul_u32_u24 %3, %3, %[a]\n\tv_mul_u32_u24 %4, %4, %[a]\n\tv_mul_u32_u24 %5, %5, %[a]\n\tv_mul_u32_u24 %6, %6, %[a]\n\tv_mul_u32_u24 %7, %7, %[a]\n\tv_mul_u32_u24 %0, %0, %[a]\n\tv_mul_u32_u24 %1, %1, %[a]\n\tv_mul_u32_u24 %2, %2, %[a]\n\tv_mul_u32_u24 %3, %3, %[a]\n\tv_mul_u32_u24 %4, %4, %[a]\n\tv_mul_u32_u24 %5, %5, %[a]\n\tv_mul_u32_u24 %6, %6, %[a]\n\tv_mul_u32_u24 %7, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[24] = t1 - t0;
}
__global__ __launch_bounds__(256) void k25(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mad_u64_u32 %[w0], vcc, %[a], %[b], %[w0]\n\tv_mad_u64_u32 %[w1], vcc, %[a], %[b], %[w1]\n\tv_mad_u64_u32 %[w2], vcc, %[a], %[b], %[w2]\n\tv_mad_u64_u32 %[w3], vcc, %[a], %[b], %[w3]\n\tv_mad_u64_u32 %[w4], vcc, %[a], %[b], %[w4]\n\tv_mad_u64_u32 %[w5], vcc, %[a], %[b], %[w5]\n\tv_mad_u64_u32 %[w6], vcc, %[a], %[b], %[w6]\n\tv_mad_u64_u32 %[w7], vcc, %[a], %[b], %[w7]\n\tv_mad_u64_u32 %[w0], vcc, %[a], %[b], %[w0]\n\tv_mad_u64_u32 %[w1], vcc, %[a], %[b], %[w1]\n\tv_mad_u64_u32 %[w2], vcc, %[a], %[b], %[w2]\n\tv_mad_u64_u32 %[w3], vcc, %[a], %[b], %[w3]\n\tv_mad_u64_u32 %[w4], vcc, %[a], %[b], %[w4]\n\tv_mad_u64_u32 %[w5], vcc, %[a], %[b], %[w5]\n\tv_mad_u64_u32 %[w6], vcc, %[a], %[b], %[w6]\n\tv_mad_u64_u32 %[w7], vcc, %[a], %[b], %[w7]\n\tv_mad_u64_u32 %[w0], vcc, %[a], %[b], %[w0]\n\tv_mad_u64_u32 %[w1], vcc, %[a], %[b], %[w1]\n\tv_mad_u64_u32 %[w2], vcc, %[a], %[b], %[w2]\n\tv_mad_u64_u32 %[w3], vcc, %[a], %[b], %[w3]\n\tv_mad_u64_u32 %[w4], vcc, %[a], %[b], %[w4]\n\tv_mad_u64_u32 %[w5], vcc, %[a], %[b], %[w5]\n\tv_mad_u64_u32 %[w6], vcc, %[a], %[b], %[w6]\n\tv_mad_u64_u32 %[w7], vcc, %[a], %[b], %[w7]\n\tv_mad_u64_u32 %[w0], vcc, %[a], %[b], %[w0]\n\tv_mad_u64_u32 %[w1], vcc, %[a], %[b], %[w1]\n\tv_mad_u64_u32 %[w2], vcc, %[a], %[b], %[w2]\n\tv_mad_u64_u32 %[w3], vcc, %[a], %[b], %[w3]\n\tv_mad_u64_u32 %[w4], vcc, %[a], %[b], %[w4]\n\tv_mad_u64_u32 %[w5], vcc, %[a], %[b], %[w5]\n\tv_mad_u64_u32 %[w6], vcc, %[a], %[b], %[w6]\n\tv_mad_u64_u32 %[w7], vcc, %[a], %[b], %[w7]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[25] = t1 - t0;
}
__global__ __launch_bounds__(256) void k26(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_cmp_lt_u32 vcc, %0, %[a]\n\tv_cmp_lt_u32 vcc, %1, %[a]\n\tv_cmp_lt_u32 vcc, %2, %[a]\n\tv_cmp_lt_u32 vcc, %3, %[a]\n\tv_cmp_lt_u32 vcc, %4, %[a]\n\tv_cmp_lt_u32 vcc, %5, %[a]\n\tv_cmp_lt_u32 vcc, %6, %[a]\n\tv_cmp_lt_u32 vcc, %7, %[a]\n\tv_cmp_lt_u32 vcc, %0, %[a]\n\tv_cmp_lt_u32 vcc, %1, %[a]\n\tv_cmp_lt_u32 vcc, %2, %[a]\n\tv_cmp_lt_u32 vcc, %3, %[a]\n\tv_cmp_lt_u32 vcc, %4, %[a]\n\tv_cmp_lt_u32 vcc, %5, %[a]\n\tv_cmp_lt_u32 vcc, %6, %[a]\n\tv_cmp_lt_u32 vcc, %7, %[a]\n\tv_cmp_lt_u32 vcc, %0, %[a]\n\tv_cmp_lt_u32 vcc, %1, %[a]\n\tv_cmp_lt_u32 vcc, %2, %[a]\n\tv_cmp_lt_u32 vcc, %3, %[a]\n\tv_cmp_lt_u32 vcc, %4, %[a]\n\tv_cmp_lt_u32 vcc, %5, %[a]\n\tv_cmp_lt_u32 vcc, %6, %[a]\n\tv_cmp_lt_u32 vcc, %7, %[a]\n\tv_cmp_lt_u32 vcc, %0, %[a]\n\tv_cmp_lt_u32 vcc, %1, %[a]\n\tv_cmp_lt_u32 vcc, %2, %[a]\n\tv_cmp_lt_u32 vcc, %3, %[a]\n\tv_cmp_lt_u32 vcc, %4, %[a]\n\tv_cmp_lt_u32 vcc, %5, %[a]\n\tv_cmp_lt_u32 vcc, %6, %[a]\n\tv_cmp_lt_u32 vcc, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[26] = t1 - t0;
}
__global__ __launch_bounds__(256) void k27(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mov_b32_dpp %0, %0 row_shr:1\n\tv_mov_b32_dpp %1, %1 row_shr:1\n\tv_mov_b32_dpp %2, %2 row_shr:1\n\tv_mov_b32_dpp %3, %3 row_shr:1\n\tv_mov_b32_dpp %4, %4 row_shr:1\n\tv_mov_b32_dpp %5, %5 row_shr:1\n\tv_mov_b32_dpp %6, %6 row_shr:1\n\tv_mov_b32_dpp %7, %7 row_shr:1\n\tv_mov_b32_dpp %0, %0 row_shr:1\n\tv_mov_b32_dpp %1, %1 row_shr:1\n\tv_mov_b32_dpp %2, %2 row_shr:1\n\tv_mov_b32_dpp %3, %3 row_shr:1\n\tv_mov_b32_dpp %4, %4 row_shr:1\n\tv_mov_b32_dpp %5, %5 row_shr:1\n\tv_mov_b32_dpp %6, %6 row_shr:1\n\tv_mov_b32_dpp %7, %7 row_shr:1\n\tv_mov_b32_dpp %0, %0 row_shr:1\n\tv_mov_b32_dpp %1, %1 row_shr:1\n\tv_mov_b32_dpp %2, %2 row_shr:1\n\tv_mov_b32_dpp %3, %3 row_shr:1\n\tv_mov_b32_dpp %4, %4 row_shr:1\n\tv_mov_b32_dpp %5, %5 row_shr:1\n\tv_mov_b32_dpp %6, %6 row_shr:1\n\tv_mov_b32_dpp %7, %7 row_shr:1\n\tv_mov_b32_dpp %0, %0 row_shr:1\n\tv_mov_b32_dpp %1, %1 row_shr:1\n\tv_mov_b32_dpp %2, %2 row_shr:1\n\tv_mov_b32_dpp %3, %3 row_shr:1\n\tv_mov_b32_dpp %4, %4 row_shr:1\n\tv_mov_b32_dpp %5, %5 row_shr:1\n\tv_mov_b32_dpp %6, %6 row_shr:1\n\tv_mov_b32_dpp %7, %7 row_shr:1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[27] = t1 - t0;
}
__global__ __launch_bounds__(256) void k28(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_subrev_co_u32 %0, vcc, %0, %[a]\n\tv_subrev_co_u32 %1, vcc, %1, %[a]\n\tv_subrev_co_u32 %2, vcc, %2, %[a]\n\tv_subrev_co_u32 %3, vcc, %3, %[a]\n\tv_subrev_co_u32 %4, vcc, %4, %[a]\n\tv_subrev_co_u32 %5, vcc, %5, %[a]\n\tv_subrev_co_u32 %6, vcc, %6, %[a]\n\tv_subrev_co_u32 %7, vcc, %7, %[a]\n\tv_subrev_co_u32 %0, vcc, %0, %[a]\n\tv_subrev_co_u32 %1, vcc, %1, %[a]\n\tv_subrev_co_u32 %2, vcc, %2, %[a]\n\tv_subrev_co_u32 %3, vcc, %3, %[a]\n\tv_subrev_co_u32 %4, vcc, %4, %[a]\n\tv_subrev_co_u32 %5, vcc, %5, %[a]\n\tv_subrev_co_u32 %6, vcc, %6, %[a]\n\tv_subrev_co_u32 %7, vcc, %7, %[a]\n\tv_subrev_co_u32 %0, vcc, %0, %[a]\n\tv_subrev_co_u32 %1, vcc, %1, %[a]\n\tv_subrev_co_u32 %2, vcc, %2, %[a]\n\tv_subrev_co_u32 %3, vcc, %3, %[a]\n\tv_subrev_co_u32 %4, vcc, %4, %[a]\n\tv_subrev_co_u32 %5, vcc, %5, %[a]\n\tv_subrev_co_u32 %6, vcc, %6, %[a]\n\tv_subrev_co_u32 %7, vcc, %7, %[a]\n\tv_subrev_co_u32 %0, vcc, %0, %[a]\n\tv_subrev_co_u32 %1, vcc, %1, %[a]\n\tv_subrev_co_u32 %2, vcc, %2, %[a]\n\tv_subrev_co_u32 %3, vcc, %3, %[a]\n\tv_subrev_co_u32 %4, vcc, %4, %[a]\n\tv_subrev_co_u32 %5, vcc, %5, %[a]\n\tv_subrev_co_u32 %6, vcc, %6, %[a]\n\tv_subrev_co_u32 %7, vcc, %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[28] = t1 - t0;
}
__global__ __launch_bounds__(256) void k29(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mov_b32 %0, %[a]\n\tv_mov_b32 %1, %[a]\n\tv_mov_b32 %2, %[a]\n\tv_mov_b32 %3, %[a]\n\tv_mov_b32 %4, %[a]\n\tv_mov_b32 %5, %[a]\n\tv_mov_b32 %6, %[a]\n\tv_mov_b32 %7, %[a]\n\tv_mov_b32 %0, %[a]\n\tv_mov_b32 %1, %[a]\n\tv_mov_b32 %2, %[a]\n\tv_mov_b32 %3, %[a]\n\tv_mov_b32 %4, %[a]\n\tv_mov_b32 %5, %[a]\n\tv_mov_b32 %6, %[a]\n\tv_mov_b32 %7, %[a]\n\tv_mov_b32 %0, %[a]\n\tv_mov_b32 %1, %[a]\n\tv_mov_b32 %2, %[a]\n\tv_mov_b32 %3, %[a]\n\tv_mov_b32 %4, %[a]\n\tv_mov_b32 %5, %[a]\n\tv_mov_b32 %6, %[a]\n\tv_mov_b32 %7, %[a]\n\tv_mov_b32 %0, %[a]\n\tv_mov_b32 %1, %[a]\n\tv_mov_b32 %2, %[a]\n\tv_mov_b32 %3, %[a]\n\tv_mov_b32 %4, %[a]\n\tv_mov_b32 %5, %[a]\n\tv_mov_b32 %6, %[a]\n\tv_mov_b32 %7, %[a]" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[29] = t1 - t0;
}
__global__ __launch_bounds__(256) void k30(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_bitop3_b32 %0, %0, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %0, %0, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %1, %1, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %2, %2, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %3, %3, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %4, %4, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %5, %5, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %6, %6, %[a], 5 bitop3:0xf1\n\tv_bitop3_b32 %7, %7, %[a], 5 bitop3:0xf1" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[30] = t1 - t0;
}
__global__ __launch_bounds__(256) void k31(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_sad_u8 %0, %[a], %[b], %0\n\tv_sad_u8 %1, %[a], %[b], %1\n\tv_sad_u8 %2, %[a], %[b], %2\n\tv_sad_u8 %3, %[a], %[b], %3\n\tv_sad_u8 %4, %[a], %[b], %4\n\tv_sad_u8 %5, %[a], %[b], %5\n\tv_sad_u8 %6, %[a], %[b], %6\n\tv_sad_u8 %7, %[a], %[b], %7\n\tv_sad_u8 %0, %[a], %[b], %0\n\tv_sad_u8 %1, %[a], %[b], %1\n\tv_sad_u8 %2, %[a], %[b], %2\n\tv_sad_u8 %3, %[a], %[b], %3\n\tv_sad_u8 %4, %[a], %[b], %4\n\tv_sad_u8 %5, %[a], %[b], %5\n\tv_sad_u8 %6, %[a], %[b], %6\n\tv_sad_u8 %7, %[a], %[b], %7\n\tv_sad_u8 %0, %[a], %[b], %0\n\tv_sad_u8 %1, %[a], %[b], %1\n\tv_sad_u8 %2, %[a], %[b], %2\n\tv_sad_u8 %3, %[a], %[b], %3\n\tv_sad_u8 %4, %[a], %[b], %4\n\tv_sad_u8 %5, %[a], %[b], %5\n\tv_sad_u8 %6, %[a], %[b], %6\n\tv_sad_u8 %7, %[a], %[b], %7\n\tv_sad_u8 %0, %[a], %[b], %0\n\tv_sad_u8 %1, %[a], %[b], %1\n\tv_sad_u8 %2, %[a], %[b], %2\n\tv_sad_u8 %3, %[a], %[b], %3\n\tv_sad_u8 %4, %[a], %[b], %4\n\tv_sad_u8 %5, %[a], %[b], %5\n\tv_sad_u8 %6, %[a], %[b], %6\n\tv_sad_u8 %7, %[a], %[b], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[31] = t1 - t0;
}
__global__ __launch_bounds__(256) void k32(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_sad_u8 %0, %[a], %[sg], %0\n\tv_sad_u8 %1, %[a], %[sg], %1\n\tv_sad_u8 %2, %[a], %[sg], %2\n\tv_sad_u8 %3, %[a], %[sg], %3\n\tv_sad_u8 %4, %[a], %[sg], %4\n\tv_sad_u8 %5, %[a], %[sg], %5\n\tv_sad_u8 %6, %[a], %[sg], %6\n\tv_sad_u8 %7, %[a], %[sg], %7\n\tv_sad_u8 %0, %[a], %[sg], %0\n\tv_sad_u8 %1, %[a], %[sg], %1\n\tv_sad_u8 %2, %[a], %[sg], %2\n\tv_sad_u8 %3, %[a], %[sg], %3\n\tv_sad_u8 %4, %[a], %[sg], %4\n\tv_sad_u8 %5, %[a], %[sg], %5\n\tv_sad_u8 %6, %[a], %[sg], %6\n\tv_sad_u8 %7, %[a], %[sg], %7\n\tv_sad_u8 %0, %[a], %[sg], %0\n\tv_sad_u8 %1, %[a], %[sg], %1\n\tv_sad_u8 %2, %[a], %[sg], %2\n\tv_sad_u8 %3, %[a], %[sg], %3\n\tv_sad_u8 %4, %[a], %[sg], %4\n\tv_sad_u8 %5, %[a], %[sg], %5\n\tv_sad_u8 %6, %[a], %[sg], %6\n\tv_sad_u8 %7, %[a], %[sg], %7\n\tv_sad_u8 %0, %[a], %[sg], %0\n\tv_sad_u8 %1, %[a], %[sg], %1\n\tv_sad_u8 %2, %[a], %[sg], %2\n\tv_sad_u8 %3, %[a], %[sg], %3\n\tv_sad_u8 %4, %[a], %[sg], %4\n\tv_sad_u8 %5, %[a], %[sg], %5\n\tv_sad_u8 %6, %[a], %[sg], %6\n\tv_sad_u8 %7, %[a], %[sg], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[32] = t1 - t0;
}
__global__ __launch_bounds__(256) void k33(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mbcnt_lo_u32_b32 %0, %[a], %0\n\tv_mbcnt_lo_u32_b32 %1, %[a], %1\n\tv_mbcnt_lo_u32_b32 %2, %[a], %2\n\tv_mbcnt_lo_u32_b32 %3, %[a], %3\n\tv_mbcnt_lo_u32_b32 %4, %[a], %4\n\tv_mbcnt_lo_u32_b32 %5, %[a], %5\n\tv_mbcnt_lo_u32_b32 %6, %[a], %6\n\tv_mbcnt_lo_u32_b32 %7, %[a], %7\n\tv_mbcnt_lo_u32_b32 %0, %[a], %0\n\tv_mbcnt_lo_u32_b32 %1, %[a], %1\n\tv_mbcnt_lo_u32_b32 %2, %[a], %2\n\tv_mbcnt_lo_u32_b32 %3, %[a], %3\n\tv_mbcnt_lo_u32_b32 %4, %[a], %4\n\tv_mbcnt_lo_u32_b32 %5, %[a], %5\n\tv_mbcnt_lo_u32_b32 %6, %[a], %6\n\tv_mbcnt_lo_u32_b32 %7, %[a], %7\n\tv_mbcnt_lo_u32_b32 %0, %[a], %0\n\tv_mbcnt_lo_u32_b32 %1, %[a], %1\n\tv_mbcnt_lo_u32_b32 %2, %[a], %2\n\tv_mbcnt_lo_u32_b32 %3, %[a], %3\n\tv_mbcnt_lo_u32_b32 %4, %[a], %4\n\tv_mbcnt_lo_u32_b32 %5, %[a], %5\n\tv_mbcnt_lo_u32_b32 %6, %[a], %6\n\tv_mbcnt_lo_u32_b32 %7, %[a], %7\n\tv_mbcnt_lo_u32_b32 %0, %[a], %0\n\tv_mbcnt_lo_u32_b32 %1, %[a], %1\n\tv_mbcnt_lo_u32_b32 %2, %[a], %2\n\tv_mbcnt_lo_u32_b32 %3, %[a], %3\n\tv_mbcnt_lo_u32_b32 %4, %[a], %4\n\tv_mbcnt_lo_u32_b32 %5, %[a], %5\n\tv_mbcnt_lo_u32_b32 %6, %[a], %6\n\tv_mbcnt_lo_u32_b32 %7, %[a], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[33] = t1 - t0;
}
__global__ __launch_bounds__(256) void k34(uint32_t* out, uint64_t* clk, uint32_t seed) {
  uint32_t v0=threadIdx.x+seed, v1=v0*3, v2=v0*5, v3=v0*7, v4=v0*9, v5=v0*11, v6=v0*13, v7=v0*15;
  uint64_t w0=v0, w1=v1, w2=v2, w3=v3, w4=v4, w5=v5, w6=v6, w7=v7, wa=(uint64_t)seed<<20;
  uint32_t a=seed*0x9e37u, b=seed^0x5555u;
  uint32_t sg = __builtin_amdgcn_readfirstlane(seed&31u);
  uint64_t sm = __builtin_amdgcn_read_exec();
  uint64_t t0 = clock64();
  for (int it = 0; it < ITERS; ++it) {
    asm volatile("v_mbcnt_hi_u32_b32 %0, %[a], %0\n\tv_mbcnt_hi_u32_b32 %1, %[a], %1\n\tv_mbcnt_hi_u32_b32 %2, %[a], %2\n\tv_mbcnt_hi_u32_b32 %3, %[a], %3\n\tv_mbcnt_hi_u32_b32 %4, %[a], %4\n\tv_mbcnt_hi_u32_b32 %5, %[a], %5\n\tv_mbcnt_hi_u32_b32 %6, %[a], %6\n\tv_mbcnt_hi_u32_b32 %7, %[a], %7\n\tv_mbcnt_hi_u32_b32 %0, %[a], %0\n\tv_mbcnt_hi_u32_b32 %1, %[a], %1\n\tv_mbcnt_hi_u32_b32 %2, %[a], %2\n\tv_mbcnt_hi_u32_b32 %3, %[a], %3\n\tv_mbcnt_hi_u32_b32 %4, %[a], %4\n\tv_mbcnt_hi_u32_b32 %5, %[a], %5\n\tv_mbcnt_hi_u32_b32 %6, %[a], %6\n\tv_mbcnt_hi_u32_b32 %7, %[a], %7\n\tv_mbcnt_hi_u32_b32 %0, %[a], %0\n\tv_mbcnt_hi_u32_b32 %1, %[a], %1\n\tv_mbcnt_hi_u32_b32 %2, %[a], %2\n\tv_mbcnt_hi_u32_b32 %3, %[a], %3\n\tv_mbcnt_hi_u32_b32 %4, %[a], %4\n\tv_mbcnt_hi_u32_b32 %5, %[a], %5\n\tv_mbcnt_hi_u32_b32 %6, %[a], %6\n\tv_mbcnt_hi_u32_b32 %7, %[a], %7\n\tv_mbcnt_hi_u32_b32 %0, %[a], %0\n\tv_mbcnt_hi_u32_b32 %1, %[a], %1\n\tv_mbcnt_hi_u32_b32 %2, %[a], %2\n\tv_mbcnt_hi_u32_b32 %3, %[a], %3\n\tv_mbcnt_hi_u32_b32 %4, %[a], %4\n\tv_mbcnt_hi_u32_b32 %5, %[a], %5\n\tv_mbcnt_hi_u32_b32 %6, %[a], %6\n\tv_mbcnt_hi_u32_b32 %7, %[a], %7" : "+v"(v0), "+v"(v1), "+v"(v2), "+v"(v3), "+v"(v4), "+v"(v5), "+v"(v6), "+v"(v7),
                 [w0] "+v"(w0), [w1] "+v"(w1), [w2] "+v"(w2), [w3] "+v"(w3), [w4] "+v"(w4), [w5] "+v"(w5), [w6] "+v"(w6), [w7] "+v"(w7)
                 : [a] "v"(a), [b] "v"(b), [sg] "s"(sg), [sm] "s"(sm), [wa] "v"(wa) : "vcc");
  }
  uint64_t t1 = clock64();
  out[blockIdx.x*256+threadIdx.x] = v0^v1^v2^v3^v4^v5^v6^v7^(uint32_t)(w0^w1^w2^w3^w4^w5^w6^w7);
  if (threadIdx.x == 0 && blockIdx.x == 0) clk[34] = t1 - t0;
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
  hipLaunchKernelGGL(k12, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k12, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[12], e0, e1);
  hipLaunchKernelGGL(k13, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k13, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[13], e0, e1);
  hipLaunchKernelGGL(k14, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k14, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[14], e0, e1);
  hipLaunchKernelGGL(k15, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k15, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[15], e0, e1);
  hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k16, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[16], e0, e1);
  hipLaunchKernelGGL(k17, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k17, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[17], e0, e1);
  hipLaunchKernelGGL(k18, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k18, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[18], e0, e1);
  hipLaunchKernelGGL(k19, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k19, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[19], e0, e1);
  hipLaunchKernelGGL(k20, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k20, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[20], e0, e1);
  hipLaunchKernelGGL(k21, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k21, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[21], e0, e1);
  hipLaunchKernelGGL(k22, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k22, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[22], e0, e1);
  hipLaunchKernelGGL(k23, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k23, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[23], e0, e1);
  hipLaunchKernelGGL(k24, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k24, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[24], e0, e1);
  hipLaunchKernelGGL(k25, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k25, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[25], e0, e1);
  hipLaunchKernelGGL(k26, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k26, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[26], e0, e1);
  hipLaunchKernelGGL(k27, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k27, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[27], e0, e1);
  hipLaunchKernelGGL(k28, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k28, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[28], e0, e1);
  hipLaunchKernelGGL(k29, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k29, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[29], e0, e1);
  hipLaunchKernelGGL(k30, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k30, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[30], e0, e1);
  hipLaunchKernelGGL(k31, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k31, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[31], e0, e1);
  hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k32, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[32], e0, e1);
  hipLaunchKernelGGL(k33, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k33, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[33], e0, e1);
  hipLaunchKernelGGL(k34, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e0); hipLaunchKernelGGL(k34, dim3(blocks), dim3(256), 0, 0, out, clk, 7u); hipEventRecord(e1); hipEventSynchronize(e1); hipEventElapsedTime(&ms[34], e0, e1);
  const char* names[] = {"bitop3_vvv", "alignbit_vvv", "alignbit_vvs", "alignbit_vvi", "add_co", "addc_co", "bcnt", "and_or", "or_vv", "lshrrev_vs", "add_vs", "lshl_add_u64", "lshrrev_vv", "lshrrev_vi", "xor_vi", "xor_vv", "add3", "lshl_add_u32", "bfe_vvv", "bcnt_vi", "cndmask_vcc", "cndmask_e64_s", "min_u32", "mul_hi_u32", "mul_u24", "mad_u64_u32", "cmp_lt_e32", "mov_dpp", "subrev_co", "mov_vv", "bitop3_vvi", "sad_u8_vvv", "sad_u8_vsv", "mbcnt_lo", "mbcnt_hi"};
  for (int n = 0; n < 35; ++n)
    printf("%-14s %.3f ms  %.2f cyc@2.4GHz per wave-instr per SIMD  (clock64 %.2f)\n", names[n], ms[n], ms[n] * 1e-3 * 2.4e9 / (4096 * 32.0 * 8.0), (double)clk[n] / (4096 * 32.0));
  return 0;
}
