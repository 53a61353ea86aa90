// Failure-schedule candidate selection: top-k seeds by
// (n_fault desc, sum_delay desc (int64), seed asc).
// Multi-level selection: each 256-thread block reduces a 2048-entry chunk to
// its best k (threshold filter + bitonic sort of the survivors in LDS); levels
// repeat until one chunk remains.
#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

constexpr uint32_t TOPK_CHUNK = 2048;

__device__ inline bool topk_better(const nmz_topk_entry &a, const nmz_topk_entry &b) {
    if (a.n_fault != b.n_fault) return a.n_fault > b.n_fault;
    if (a.sum_delay_ns != b.sum_delay_ns) return a.sum_delay_ns > b.sum_delay_ns;
    return a.seed < b.seed;
}

__device__ inline nmz_topk_entry topk_sentinel() {
    nmz_topk_entry e;
    e.seed = UINT64_MAX;
    e.sum_delay_ns = INT64_MIN;
    e.n_fault = 0;
    e.first_fault = NMZ_NONE;
    return e;
}

// bitonic sort (best first) of the first `n` entries of s (n a power of two)
__device__ void bitonic_sort_n(nmz_topk_entry *s, uint32_t n) {
    for (uint32_t size = 2; size <= n; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < n / 2; t += blockDim.x) {
                uint32_t i = 2 * t - (t & (stride - 1));
                uint32_t j = i + stride;
                bool best_first = ((i & size) == 0);
                nmz_topk_entry a = s[i], b = s[j];
                bool swap = best_first ? topk_better(b, a) : topk_better(a, b);
                if (swap) {
                    s[i] = b;
                    s[j] = a;
                }
            }
        }
    }
    __syncthreads();
}

constexpr uint32_t TOPK_THREADS = 256;
constexpr uint32_t TOPK_PER_THREAD = TOPK_CHUNK / TOPK_THREADS;

// Chunk top-k by threshold filtering. Each thread's best entry is a "winner";
// the k-th best winner T is a lower bound of the chunk's k-th best entry (k
// distinct entries are >= T), so only entries >= T can be in the chunk's
// top-k. The survivors (typically ~k) are compacted in LDS and sorted.
template <bool FROM_STATS>
__global__ __launch_bounds__(TOPK_THREADS) void k_topk_chunk(const void *__restrict__ src, uint64_t n,
                                                              uint64_t seed0, uint32_t k,
                                                              nmz_topk_entry *__restrict__ out) {
    __shared__ nmz_topk_entry cand[TOPK_CHUNK];
    __shared__ nmz_topk_entry win[TOPK_THREADS];
    __shared__ uint32_t ncand;
    const uint32_t t = threadIdx.x;
    const uint64_t base = (uint64_t)blockIdx.x * TOPK_CHUNK;
    nmz_topk_entry e[TOPK_PER_THREAD];
    nmz_topk_entry best = topk_sentinel();
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        const uint64_t i = base + (uint64_t)r * TOPK_THREADS + t;
        nmz_topk_entry x = topk_sentinel();
        if (i < n) {
            if (FROM_STATS) {
                const nmz_sched_stats st = static_cast<const nmz_sched_stats *>(src)[i];
                x.seed = seed0 + i;
                x.sum_delay_ns = (int64_t)st.sum_delay_ns;
                x.n_fault = st.n_fault;
                x.first_fault = st.first_fault;
            } else {
                x = static_cast<const nmz_topk_entry *>(src)[i];
            }
        }
        e[r] = x;
        if (topk_better(x, best)) best = x;
    }
    win[t] = best;
    if (t == 0) ncand = 0;
    bitonic_sort_n(win, TOPK_THREADS);
    const nmz_topk_entry T = win[k - 1];
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        if (!topk_better(T, e[r])) cand[atomicAdd(&ncand, 1u)] = e[r];  // e >= T
    }
    __syncthreads();
    const uint32_t c = ncand;
    uint32_t np = 2;
    while (np < c) np <<= 1;
    for (uint32_t i = c + t; i < np; i += TOPK_THREADS) cand[i] = topk_sentinel();
    bitonic_sort_n(cand, np);
    for (uint32_t i = t; i < k; i += TOPK_THREADS)
        out[(uint64_t)blockIdx.x * k + i] = i < c ? cand[i] : topk_sentinel();
}

uint64_t topk_scratch_entries(uint64_t n, uint32_t k) {
    if (k == 0) return 0;
    uint64_t blocks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    if (blocks == 0) blocks = 1;
    return 2 * blocks * k + 2 * TOPK_CHUNK;
}

// Writes the best k entries to d_out (device). scratch must hold
// topk_scratch_entries(n, k) entries.
int topk_select(hipStream_t st, const nmz_sched_stats *d_stats, uint64_t n, uint64_t seed0, uint32_t k,
                nmz_topk_entry *d_scratch, nmz_topk_entry *d_out) {
    if (k == 0) return NMZ_OK;
    NMZ_CHECK(k <= TOPK_THREADS, "top-k supports k <= 256");
    uint64_t blocks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    if (blocks == 0) blocks = 1;
    nmz_topk_entry *a = d_scratch, *b = d_scratch + blocks * k;
    hipLaunchKernelGGL(k_topk_chunk<true>, dim3((unsigned)blocks), dim3(TOPK_THREADS), 0, st, d_stats, n, seed0, k,
                       blocks == 1 ? d_out : a);
    uint64_t cur = blocks * k;
    while (blocks > 1) {
        blocks = (cur + TOPK_CHUNK - 1) / TOPK_CHUNK;
        hipLaunchKernelGGL(k_topk_chunk<false>, dim3((unsigned)blocks), dim3(TOPK_THREADS), 0, st, a, cur, 0, k,
                           blocks == 1 ? d_out : b);
        cur = blocks * k;
        nmz_topk_entry *tmp = a;
        a = b;
        b = tmp;
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz

using namespace nmz;

extern "C" int nmz_topk_select_dev(nmz_ctx *ctx, const nmz_sched_stats *d_stats, uint64_t n, uint64_t seed0,
                                   uint32_t k, nmz_topk_entry *d_out, void *stream) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (k == 0) return NMZ_OK;
    NMZ_TRY(ctx->buf[5].ensure(topk_scratch_entries(n, k) * sizeof(nmz_topk_entry) + 256));
    return topk_select(stream ? (hipStream_t)stream : ctx->stream, d_stats, n, seed0, k,
                       ctx->buf[5].as<nmz_topk_entry>(), d_out);
}
