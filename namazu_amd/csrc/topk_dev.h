// Device-side top-k pieces shared by k_topk_chunk (topk.hip) and the fused
// merge + selection of the replayable sweep (replayable.hip).
#pragma once
#include "nmz_common.h"

namespace nmz {

constexpr uint32_t TOPK_CHUNK = 2048;
constexpr uint32_t TOPK_THREADS = 256;
constexpr uint32_t TOPK_PER_THREAD = TOPK_CHUNK / TOPK_THREADS;
constexpr uint32_t TOPK_RANK_MAX = 512;   // survivors ranked by counting; more -> bitonic sort
constexpr uint32_t TOPK_MERGE_SLOTS = 4096;  // LDS entries per merge block (96 KiB)

__device__ inline bool topk_better(const nmz_topk_entry &a, const nmz_topk_entry &b) {
    if (a.n_fault != b.n_fault) return a.n_fault > b.n_fault;
    if (a.sum_delay_ns != b.sum_delay_ns) return a.sum_delay_ns > b.sum_delay_ns;
    return a.seed < b.seed;
}

// strict total order: topk_better, then chunk position (equal entries: sentinels)
__device__ inline bool topk_before(const nmz_topk_entry &a, uint32_t ia, const nmz_topk_entry &b, uint32_t ib) {
    if (a.n_fault != b.n_fault) return a.n_fault > b.n_fault;
    if (a.sum_delay_ns != b.sum_delay_ns) return a.sum_delay_ns > b.sum_delay_ns;
    if (a.seed != b.seed) return a.seed < b.seed;
    return ia < ib;
}

__device__ inline bool topk_is_sentinel(const nmz_topk_entry &x) {
    return x.seed == UINT64_MAX && x.sum_delay_ns == INT64_MIN && x.n_fault == 0;
}

__device__ inline nmz_topk_entry topk_sentinel() {
    nmz_topk_entry e;
    e.seed = UINT64_MAX;
    e.sum_delay_ns = INT64_MIN;
    e.n_fault = 0;
    e.first_fault = NMZ_NONE;
    return e;
}

// Coarse key: a better than b => coarse(a) >= coarse(b). n_fault in the top 16
// bits (saturated: every entry with >= 0xffff faults maps to the maximum key),
// then the top 48 bits of the order-preserving (sign-flipped) sum.
__device__ inline uint64_t topk_coarse(const nmz_topk_entry &x) {
    if (x.n_fault >= 0xffffu) return UINT64_MAX;
    const uint64_t bs = (uint64_t)x.sum_delay_ns ^ (1ull << 63);
    return ((uint64_t)x.n_fault << 48) | (bs >> 16);
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

struct TopkShared {
    nmz_topk_entry cand[TOPK_CHUNK];
    uint32_t cidx[TOPK_CHUNK];
    uint64_t wkey[TOPK_THREADS];
    uint64_t tau;
    uint32_t ncand;
};

// The block's best k of its TOPK_CHUNK entries, sorted, to o[0..k). Thread t holds entries e[r] at chunk
// positions r * TOPK_THREADS + t (sentinels for unused positions); blockDim.x == TOPK_THREADS.
// A 64-bit coarse key (monotone in the order, not strict) gives a threshold tau = the k-th largest
// per-thread maximum: at least k entries reach it, and every member of the chunk's top-k does. The
// survivors (typically ~k) are ranked exactly by counting and written to their slot.
__device__ inline void topk_block_select(const nmz_topk_entry (&e)[TOPK_PER_THREAD], uint32_t k,
                                         nmz_topk_entry *__restrict__ o, TopkShared &sh) {
    const uint32_t t = threadIdx.x;
    uint64_t ck[TOPK_PER_THREAD];
    uint64_t wk = 0;
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        ck[r] = topk_coarse(e[r]);
        wk = ck[r] > wk ? ck[r] : wk;
    }
    sh.wkey[t] = wk;
    if (t == 0) sh.ncand = 0;
    __syncthreads();
    // tau = k-th largest per-thread maximum (with multiplicity)
    uint32_t gt = 0, ge = 0;
#pragma unroll 8
    for (uint32_t j = 0; j < TOPK_THREADS; ++j) {
        const uint64_t w = sh.wkey[j];
        gt += w > wk ? 1u : 0u;
        ge += w >= wk ? 1u : 0u;
    }
    if (gt < k && k <= ge) sh.tau = wk;  // every writer writes the same value
    __syncthreads();
    const uint64_t tau = sh.tau;
    // Sentinels (padding) rank after every real entry, so they never compete: they are left out
    // of the candidates and fill the slots past the real ones (a block of padding alone would
    // otherwise send 2048 equal entries to the bitonic sort).
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        if (ck[r] >= tau && !topk_is_sentinel(e[r])) {
            const uint32_t c = atomicAdd(&sh.ncand, 1u);
            sh.cand[c] = e[r];
            sh.cidx[c] = r * TOPK_THREADS + t;
        }
    }
    __syncthreads();
    const uint32_t c = sh.ncand;  // >= k unless the block holds fewer than k real entries
    for (uint32_t i = c + t; i < k; i += TOPK_THREADS) o[i] = topk_sentinel();
    if (c <= TOPK_RANK_MAX) {
        for (uint32_t i = t; i < c; i += TOPK_THREADS) {
            const nmz_topk_entry x = sh.cand[i];
            const uint32_t xi = sh.cidx[i];
            uint32_t rk = 0;
            for (uint32_t j = 0; j < c; ++j) rk += topk_before(sh.cand[j], sh.cidx[j], x, xi) ? 1u : 0u;
            if (rk < k) o[rk] = x;
        }
        return;
    }
    uint32_t np = 2;
    while (np < c) np <<= 1;
    for (uint32_t i = c + t; i < np; i += TOPK_THREADS) sh.cand[i] = topk_sentinel();
    bitonic_sort_n(sh.cand, np);
    for (uint32_t i = t; i < k && i < c; i += TOPK_THREADS) o[i] = sh.cand[i];
}

}  // namespace nmz
