// Direction check for gfx9 DPP wavefront shifts (wave_shl:1 = 0x130, wave_shr:1 = 0x138).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(int *o) {
    int x = threadIdx.x + 100;
    o[threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x130, 0xf, 0xf, false);
    o[64 + threadIdx.x] = __builtin_amdgcn_update_dpp(-1, x, 0x138, 0xf, 0xf, false);
}
int main() {
    int *o;
    (void)hipMallocManaged(&o, 128 * 4);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, o);
    (void)hipDeviceSynchronize();
    printf("wave_shl1: lane0=%d lane1=%d lane62=%d lane63=%d\n", o[0], o[1], o[62], o[63]);
    printf("wave_shr1: lane0=%d lane1=%d lane62=%d lane63=%d\n", o[64], o[65], o[126], o[127]);
    return 0;
}
