// Failure-schedule candidate selection: top-k seeds by
// (n_fault desc, sum_delay desc (int64), seed asc).
// Two-level selection: each 256-thread block bitonic-sorts a 2048-entry chunk
// in LDS and keeps its best k; levels repeat until one chunk remains.
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

// sort `s` (TOPK_CHUNK entries in LDS) best-first
__device__ void bitonic_sort_chunk(nmz_topk_entry *s) {
    for (uint32_t size = 2; size <= TOPK_CHUNK; size <<= 1) {
        for (uint32_t stride = size >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (uint32_t t = threadIdx.x; t < TOPK_CHUNK / 2; t += blockDim.x) {
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

// level 0: from stats (seed value = seed0 + index)
__global__ __launch_bounds__(256) void k_topk_from_stats(const nmz_sched_stats *__restrict__ stats,
                                                         uint64_t n, uint64_t seed0, uint32_t k,
                                                         nmz_topk_entry *__restrict__ out) {
    __shared__ nmz_topk_entry s[TOPK_CHUNK];
    uint64_t base = (uint64_t)blockIdx.x * TOPK_CHUNK;
    for (uint32_t t = threadIdx.x; t < TOPK_CHUNK; t += blockDim.x) {
        uint64_t i = base + t;
        nmz_topk_entry e = topk_sentinel();
        if (i < n) {
            const nmz_sched_stats st = stats[i];
            e.seed = seed0 + i;
            e.sum_delay_ns = (int64_t)st.sum_delay_ns;
            e.n_fault = st.n_fault;
            e.first_fault = st.first_fault;
        }
        s[t] = e;
    }
    bitonic_sort_chunk(s);
    for (uint32_t t = threadIdx.x; t < k; t += blockDim.x) out[(uint64_t)blockIdx.x * k + t] = s[t];
}

// level >= 1: from candidate entries
__global__ __launch_bounds__(256) void k_topk_merge(const nmz_topk_entry *__restrict__ in, uint64_t n,
                                                    uint32_t k, nmz_topk_entry *__restrict__ out) {
    __shared__ nmz_topk_entry s[TOPK_CHUNK];
    uint64_t base = (uint64_t)blockIdx.x * TOPK_CHUNK;
    for (uint32_t t = threadIdx.x; t < TOPK_CHUNK; t += blockDim.x) {
        uint64_t i = base + t;
        s[t] = (i < n) ? in[i] : topk_sentinel();
    }
    bitonic_sort_chunk(s);
    for (uint32_t t = threadIdx.x; t < k; t += blockDim.x) out[(uint64_t)blockIdx.x * k + t] = s[t];
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
    NMZ_CHECK(k <= TOPK_CHUNK / 2, "top-k supports k <= 1024");
    uint64_t blocks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    if (blocks == 0) blocks = 1;
    nmz_topk_entry *a = d_scratch, *b = d_scratch + blocks * k;
    hipLaunchKernelGGL(k_topk_from_stats, dim3((unsigned)blocks), dim3(256), 0, st, d_stats, n, seed0, k,
                       blocks == 1 ? d_out : a);
    uint64_t cur = blocks * k;
    while (blocks > 1) {
        blocks = (cur + TOPK_CHUNK - 1) / TOPK_CHUNK;
        hipLaunchKernelGGL(k_topk_merge, dim3((unsigned)blocks), dim3(256), 0, st, a, cur, k,
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
