// Do streams share hardware queues?  N streams each get one spinning single-block kernel of ~200 us; if the
// streams run on distinct hardware queues the N kernels overlap (~200 us in all), streams that share a queue
// run one after another.  usage: stream_queues <plain|cumask|prio> <max streams>
// build: hipcc --offload-arch=gfx950 -O2 -o stream_queues stream_queues.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

__global__ void k_spin(uint64_t ticks, uint64_t *out) {
    const uint64_t t0 = wall_clock64();
    uint64_t t = t0;
    while (t - t0 < ticks) t = wall_clock64();
    if (threadIdx.x == 0) out[blockIdx.x] = t - t0;
}

#define CK(x)                                                                   \
    do {                                                                        \
        hipError_t e_ = (x);                                                    \
        if (e_ != hipSuccess) {                                                 \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));        \
            return 1;                                                           \
        }                                                                       \
    } while (0)

int main(int argc, char **argv) {
    const char *mode = argc > 1 ? argv[1] : "plain";
    const int max_n = argc > 2 ? std::atoi(argv[2]) : 8;
    int rate_khz = 0;
    CK(hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0));
    const uint64_t ticks = (uint64_t)rate_khz * 200 / 1000;  // 200 us
    uint64_t *d_out;
    CK(hipMalloc(&d_out, 64 * sizeof(uint64_t)));
    std::vector<hipStream_t> st(max_n);
    std::vector<uint32_t> mask(8, 0xffffffffu);
    int lo = 0, hi = 0;
    CK(hipDeviceGetStreamPriorityRange(&lo, &hi));
    for (int i = 0; i < max_n; ++i) {
        if (!std::strcmp(mode, "cumask"))
            CK(hipExtStreamCreateWithCUMask(&st[i], (uint32_t)mask.size(), mask.data()));
        else if (!std::strcmp(mode, "prio"))
            CK(hipStreamCreateWithPriority(&st[i], hipStreamNonBlocking, i % 2 ? lo : hi));
        else
            CK(hipStreamCreateWithFlags(&st[i], hipStreamNonBlocking));
    }
    std::printf("mode %s wall clock %d kHz priority range %d..%d\n", mode, rate_khz, lo, hi);
    for (int n = 1; n <= max_n; ++n) {
        std::vector<double> us;
        for (int rep = 0; rep < 7; ++rep) {
            CK(hipDeviceSynchronize());
            const auto t0 = std::chrono::steady_clock::now();
            for (int i = 0; i < n; ++i) hipLaunchKernelGGL(k_spin, dim3(1), dim3(64), 0, st[i], ticks, d_out + i);
            CK(hipGetLastError());
            CK(hipDeviceSynchronize());
            us.push_back(std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t0).count());
        }
        std::sort(us.begin(), us.end());
        std::printf("streams %d: %.0f us (x%.2f of one kernel)\n", n, us[3], us[3] / 200.0);
    }
    for (auto s : st) CK(hipStreamDestroy(s));
    CK(hipFree(d_out));
    return 0;
}
