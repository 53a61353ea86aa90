// Device-side top-k pieces shared by k_topk_chunk (topk.hip) and the fused
// merge + selection of the replayable sweep (replayable.hip).
#pragma once
#include "nmz_common.h"

namespace nmz {

constexpr uint32_t TOPK_CHUNK = 2048;
constexpr uint32_t TOPK_THREADS = 256;
constexpr uint32_t TOPK_PER_THREAD = TOPK_CHUNK / TOPK_THREADS;
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

// LDS of one selection block: candidates up to TOPK_LDS_CAND (the coarse threshold leaves ~k of them unless
// many entries tie on the coarse key), so the block fits beside a K1 order-query workgroup (<= 45 KB left on a CU)
constexpr uint32_t TOPK_LDS_CAND = 512;
struct TopkShared {
    nmz_topk_entry cand[TOPK_LDS_CAND];
    uint32_t cidx[TOPK_LDS_CAND];
    uint64_t wkey[TOPK_THREADS];
    uint64_t tau;
    uint32_t ncand;
    uint32_t win;
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
    // of the candidates and fill the slots past the real ones. Candidates are counted in full but stored only
    // while they fit the LDS list.
#pragma unroll
    for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r) {
        if (ck[r] >= tau && !topk_is_sentinel(e[r])) {
            const uint32_t c = atomicAdd(&sh.ncand, 1u);
            if (c < TOPK_LDS_CAND) {
                sh.cand[c] = e[r];
                sh.cidx[c] = r * TOPK_THREADS + t;
            }
        }
    }
    __syncthreads();
    const uint32_t c = sh.ncand;  // >= k unless the block holds fewer than k real entries
    for (uint32_t i = c + t; i < k; i += TOPK_THREADS) o[i] = topk_sentinel();
    if (c <= TOPK_LDS_CAND) {
        for (uint32_t i = t; i < c; i += TOPK_THREADS) {
            const nmz_topk_entry x = sh.cand[i];
            const uint32_t xi = sh.cidx[i];
            uint32_t rk = 0;
            for (uint32_t j = 0; j < c; ++j) rk += topk_before(sh.cand[j], sh.cidx[j], x, xi) ? 1u : 0u;
            if (rk < k) o[rk] = x;
        }
        return;
    }
    // Many entries tie on the coarse key (e.g. equal sums): take the best k one at a time, each round a block
    // reduction over every thread's best unused candidate.
    uint32_t used = 0;
    for (uint32_t i = 0; i < k && i < c; ++i) {
        int br = -1;
#pragma unroll
        for (uint32_t r = 0; r < TOPK_PER_THREAD; ++r)
            if (!((used >> r) & 1u) && ck[r] >= tau && !topk_is_sentinel(e[r]) &&
                (br < 0 || topk_before(e[r], r * TOPK_THREADS + t, e[br], (uint32_t)br * TOPK_THREADS + t)))
                br = (int)r;
        sh.cand[t] = br >= 0 ? e[br] : topk_sentinel();
        sh.cidx[t] = br >= 0 ? (uint32_t)br * TOPK_THREADS + t : UINT32_MAX;
        __syncthreads();
        for (uint32_t st = TOPK_THREADS / 2; st; st >>= 1) {
            if (t < st && topk_before(sh.cand[t + st], sh.cidx[t + st], sh.cand[t], sh.cidx[t])) {
                sh.cand[t] = sh.cand[t + st];
                sh.cidx[t] = sh.cidx[t + st];
            }
            __syncthreads();
        }
        const uint32_t win = sh.cidx[0];
        if (t == 0) o[i] = sh.cand[0];
        if (win % TOPK_THREADS == t) used |= 1u << (win / TOPK_THREADS);
        __syncthreads();
    }
}

}  // namespace nmz
