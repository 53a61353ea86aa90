// Failure-schedule candidate selection: top-k seeds by
// (n_fault desc, sum_delay desc (int64), seed asc).
//
// Two kernels, no full sorts:
//  1. k_topk_chunk: a 256-thread block reduces a 2048-entry chunk of the
//     stats to its best k, sorted. A 64-bit coarse key (monotone in the
//     order, not strict) gives a threshold tau = the k-th largest per-thread
//     maximum: at least k entries reach it, and every member of the chunk's
//     top-k does. The survivors (typically ~k) are ranked exactly by counting
//     and written to their slot.
//  2. k_topk_merge_wave (k <= 64): a 1024-thread block merges 32 sorted lists,
//     one list per wave in registers (lane l = entry l), pairwise bitonic merges
//     with cross-lane shuffles and 4 barriers. k_topk_merge (k > 64): a block
//     merges up to 32 sorted lists into one sorted list
//     of k by a tree of bitonic merges in LDS (elementwise best of A[i] and
//     B[kp-1-i] is a bitonic sequence holding the top kp of both; log2(kp)
//     half-cleaner stages sort it). Levels repeat until one list remains.
#include "nmz_common.h"
#include "nmz_internal.h"
#include "topk_dev.h"

namespace nmz {

__global__ __launch_bounds__(TOPK_THREADS) void k_topk_chunk(const nmz_sched_stats *__restrict__ stats, uint64_t n,
                                                              uint64_t seed0, uint32_t k,
                                                              nmz_topk_entry *__restrict__ out) {
    __shared__ TopkShared sh;
    const uint64_t base = (uint64_t)blockIdx.x * TOPK_CHUNK;
    nmz_topk_entry e[TOPK_PER_THREAD];
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        const uint64_t i = base + (uint64_t)r * TOPK_THREADS + threadIdx.x;
        nmz_topk_entry x = topk_sentinel();
        if (i < n) {
            const nmz_sched_stats st = stats[i];
            x.seed = seed0 + i;
            x.sum_delay_ns = (int64_t)st.sum_delay_ns;
            x.n_fault = st.n_fault;
            x.first_fault = st.first_fault;
        }
        e[r] = x;
    }
    topk_block_select(e, k, out + (uint64_t)blockIdx.x * k, sh);
}

// Merge `lpb` consecutive sorted lists of k entries (kp = next pow2 >= k,
// lpb * kp <= TOPK_MERGE_SLOTS) into one sorted list of k. Lists past n_lists
// are sentinels.
__global__ __launch_bounds__(TOPK_THREADS) void k_topk_merge(const nmz_topk_entry *__restrict__ in,
                                                              uint32_t n_lists, uint32_t k, uint32_t lkp,
                                                              uint32_t lpb, nmz_topk_entry *__restrict__ out) {
    // kp = 2^lkp: index math by shifts and masks (runtime divisions cost ~40 VALU each)
    const uint32_t kp = 1u << lkp, kmask = kp - 1, lh = lkp ? lkp - 1 : 0, hmask = (kp >> 1) - 1;
    __shared__ nmz_topk_entry s[TOPK_MERGE_SLOTS];
    const uint32_t t = threadIdx.x;
    const uint32_t l0 = blockIdx.x * lpb;
    for (uint32_t i = t; i < lpb * kp; i += TOPK_THREADS) {
        const uint32_t l = l0 + (i >> lkp), j = i & kmask;
        s[i] = (l < n_lists && j < k) ? in[(uint64_t)l * k + j] : topk_sentinel();
    }
    for (uint32_t w = 1; w < lpb; w <<= 1) {  // merge list pairs (a, a + w), a % 2w == 0
        const uint32_t pairs = lpb / (2 * w);
        __syncthreads();
        for (uint32_t i = t; i < pairs * kp; i += TOPK_THREADS) {
            const uint32_t a = (i >> lkp) * 2 * w, j = i & kmask;
            nmz_topk_entry &x = s[a * kp + j];
            const nmz_topk_entry y = s[(a + w) * kp + (kp - 1 - j)];
            if (topk_better(y, x)) x = y;
        }
        for (uint32_t stride = kp >> 1; stride > 0; stride >>= 1) {
            __syncthreads();
            for (uint32_t i = t; i < pairs * (kp >> 1); i += TOPK_THREADS) {
                const uint32_t a = (i >> lh) * 2 * w, q = i & hmask;
                const uint32_t p = 2 * q - (q & (stride - 1));
                nmz_topk_entry &x = s[a * kp + p];
                nmz_topk_entry &y = s[a * kp + p + stride];
                if (topk_better(y, x)) {
                    const nmz_topk_entry tmp = x;
                    x = y;
                    y = tmp;
                }
            }
        }
    }
    __syncthreads();
    for (uint32_t j = t; j < k; j += TOPK_THREADS) out[(uint64_t)blockIdx.x * k + j] = s[j];
}

// ---- k <= 64: list merges in registers, one list per wave (lane l holds entry l) ----
__device__ __forceinline__ nmz_topk_entry shfl_xor_entry(const nmz_topk_entry &x, uint32_t s) {
    nmz_topk_entry y;
    y.seed = __shfl_xor(x.seed, s, 64);
    y.sum_delay_ns = __shfl_xor(x.sum_delay_ns, s, 64);
    y.n_fault = __shfl_xor(x.n_fault, s, 64);
    y.first_fault = __shfl_xor(x.first_fault, s, 64);
    return y;
}

// x: sorted list A (best first) over lanes 0..kp-1; yr: list B reversed (lane l holds B[kp-1-l]).
// Elementwise best is a bitonic sequence holding the top kp of A u B; half-cleaners sort it.
__device__ __forceinline__ void wave_merge(nmz_topk_entry &x, const nmz_topk_entry &yr, uint32_t kp, uint32_t lane) {
    if (topk_better(yr, x)) x = yr;
    for (uint32_t st = kp >> 1; st > 0; st >>= 1) {
        const nmz_topk_entry p = shfl_xor_entry(x, st);
        const bool lower = (lane & st) == 0;
        if (lower ? topk_better(p, x) : topk_better(x, p)) x = p;
    }
}

constexpr uint32_t TOPK_WAVE_LISTS = 32;  // lists merged per 1024-thread block

// Merge up to 32 consecutive sorted lists of k (kp = pow2 >= k <= 64) into one: round 1 merges list pairs
// straight from global memory (one pair per wave), later rounds pair wave w with wave w + n through one LDS
// slot per wave (24 KB, so a block fits beside a K1 order-query workgroup); 5 rounds, 4 barriers.
__global__ __launch_bounds__(1024) void k_topk_merge_wave(const nmz_topk_entry *__restrict__ in, uint32_t n_lists,
                                                          uint32_t k, uint32_t kp,
                                                          nmz_topk_entry *__restrict__ out) {
    __shared__ nmz_topk_entry slot[TOPK_WAVE_LISTS / 2][64];
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const uint64_t l0 = (uint64_t)blockIdx.x * TOPK_WAVE_LISTS;
    auto load = [&](uint64_t l, uint32_t j) {
        return (l < n_lists && j < k) ? in[l * k + j] : topk_sentinel();
    };
    // round 1: wave w merges lists 2w, 2w+1
    nmz_topk_entry x = lane < kp ? load(l0 + 2 * w, lane) : topk_sentinel();
    {
        const nmz_topk_entry yr = lane < kp ? load(l0 + 2 * w + 1, kp - 1 - lane) : topk_sentinel();
        wave_merge(x, yr, kp, lane);
        slot[w][lane] = x;
    }
    // rounds 2..5: wave w < n merges wave w + n's list (slots >= n are not written in that round)
    for (uint32_t n = TOPK_WAVE_LISTS / 4; n >= 1; n >>= 1) {
        __syncthreads();
        if (w < n) {
            const nmz_topk_entry yr = lane < kp ? slot[w + n][kp - 1 - lane] : topk_sentinel();
            wave_merge(x, yr, kp, lane);
            slot[w][lane] = x;
        }
    }
    if (w == 0 && lane < k) out[(uint64_t)blockIdx.x * k + lane] = x;
}

static uint32_t pow2_at_least(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

uint64_t topk_scratch_entries(uint64_t n, uint32_t k) {
    if (k == 0) return 0;
    uint64_t blocks = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    if (blocks == 0) blocks = 1;
    return 2 * blocks * k + 2 * TOPK_CHUNK;
}

// Merges n_lists sorted lists of k entries (in `a`; `b` is scratch of the same size) into the best k,
// written to d_out. Both buffers are overwritten.
int topk_merge_lists(hipStream_t st, nmz_topk_entry *a, nmz_topk_entry *b, uint64_t lists, uint32_t k,
                     nmz_topk_entry *d_out) {
    const uint32_t kp = pow2_at_least(k);
    const uint32_t lkp = (uint32_t)__builtin_ctz(kp);
    const uint32_t lpb = std::min<uint32_t>(32, TOPK_MERGE_SLOTS / kp);
    if (lists == 1) {
        NMZ_HIP(hipMemcpyAsync(d_out, a, (size_t)k * sizeof(nmz_topk_entry), hipMemcpyDeviceToDevice, st));
        return NMZ_OK;
    }
    while (kp <= 64 && lists > 1) {
        const uint64_t nb = (lists + TOPK_WAVE_LISTS - 1) / TOPK_WAVE_LISTS;
        hipLaunchKernelGGL(k_topk_merge_wave, dim3((unsigned)nb), dim3(1024), 0, st, a, (uint32_t)lists, k, kp,
                           nb == 1 ? d_out : b);
        lists = nb;
        nmz_topk_entry *tmp = a;
        a = b;
        b = tmp;
    }
    while (lists > 1) {
        const uint64_t nb = (lists + lpb - 1) / lpb;
        hipLaunchKernelGGL(k_topk_merge, dim3((unsigned)nb), dim3(TOPK_THREADS), 0, st, a, (uint32_t)lists, k, lkp,
                           lpb, nb == 1 ? d_out : b);
        lists = nb;
        nmz_topk_entry *tmp = a;
        a = b;
        b = tmp;
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// Writes the best k entries to d_out (device). scratch must hold
// topk_scratch_entries(n, k) entries.
int topk_select(hipStream_t st, const nmz_sched_stats *d_stats, uint64_t n, uint64_t seed0, uint32_t k,
                nmz_topk_entry *d_scratch, nmz_topk_entry *d_out) {
    if (k == 0) return NMZ_OK;
    NMZ_CHECK(k <= TOPK_THREADS, "top-k supports k <= 256");
    uint64_t lists = (n + TOPK_CHUNK - 1) / TOPK_CHUNK;
    if (lists == 0) lists = 1;
    NMZ_CHECK(lists < (1ull << 31), "too many seeds for one top-k selection");
    nmz_topk_entry *a = d_scratch, *b = d_scratch + lists * k;
    hipLaunchKernelGGL(k_topk_chunk, dim3((unsigned)lists), dim3(TOPK_THREADS), 0, st, d_stats, n, seed0, k,
                       lists == 1 ? d_out : a);
    NMZ_HIP(hipGetLastError());
    if (lists == 1) return NMZ_OK;
    return topk_merge_lists(st, a, b, lists, k, d_out);
}

}  // namespace nmz

using namespace nmz;

extern "C" int nmz_topk_merge_dev(nmz_ctx *ctx, nmz_topk_entry *d_lists, uint64_t n_lists, uint32_t k,
                                  nmz_topk_entry *d_scratch, nmz_topk_entry *d_out, void *stream) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(k <= 256, "k must be <= 256");
    if (k == 0 || n_lists == 0) return NMZ_OK;
    NMZ_CHECK(d_lists && d_scratch && d_out, "NULL argument");
    NMZ_CHECK(n_lists < (1ULL << 31), "too many lists");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return topk_merge_lists(stream ? (hipStream_t)stream : ctx->stream, d_lists, d_scratch, n_lists, k, d_out);
}

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
