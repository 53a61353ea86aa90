#include <cstdlib>
// K3 -- banded Levenshtein over event-hash sequences + all-pairs k-NN.
//
// ED_w(a,b) = min(D(n,m), w+1), D restricted to |i-j| <= w (outside = +inf).
// Distance 0 <=> element-wise equal traces (SingleTrace.Equals,
// util/trace/trace.go:29-31); see DESIGN.md section 4.
//
// Fast path (k_ed_tile<W>), MI355X-first:
//  * symbols are remapped to dense 16-bit ids (exact: equality preserved);
//  * one lane per candidate trace b and TWO query traces (q1,q2) per wave,
//    packed in the lo/hi u16 halves of every register, so each packed VALU
//    op advances two DP cells; the band row (2W+1 cells) and a sliding window
//    of 2W+R candidate symbols live in VGPRs -- no cross-lane traffic, all 64
//    lanes busy (a wave-per-pair anti-diagonal mapping keeps at most w+1 of
//    64 lanes busy per step for w = 32);
//  * query symbols are wave-uniform scalar loads; candidate symbols come
//    from a lane-interleaved layout ([group][pos][64 lanes], one coalesced
//    128-B line per position), prefetched one row block ahead;
//  * Ukkonen cut-off: the band minimum of a row never decreases, so once it
//    exceeds W for both halves of every lane the wave stops (result W+1).
// Results go straight into per-trace top-k lists (u64 keys dist<<32|id,
// cascade atomicMin insertion: lock-free and order-independent).
//
// Generic path (k_ed_generic): one thread per pair, any band, u64 symbols,
// band row in global scratch. Used for nmz_ed_pairs and as the fallback.
#include <algorithm>
#include <chrono>
#include <thread>
#include <unordered_map>
#include <vector>

#include <map>

#include <hipcub/hipcub.hpp>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));

constexpr uint16_t CAND_PAD = 0xffff;  // candidate symbol past its end (never a real id)
constexpr uint16_t QUERY_PAD = 0xfffe; // query symbol past its end
constexpr uint16_t INF16 = 0x7f00;     // +inf for u16 DP cells (grows by < W before leaving the band)
constexpr int ED_R = 8;                // rows per unrolled block
constexpr uint32_t MAX_FAST_LEN = 0x7000;
constexpr uint32_t MAX_FAST_SYMBOLS = 0xfffd;

__device__ __forceinline__ u16x2 pk_min(u16x2 a, u16x2 b) { return __builtin_elementwise_min(a, b); }
__device__ __forceinline__ u16x2 splat(uint16_t v) { return u16x2{v, v}; }
__device__ __forceinline__ u16x2 as_pk(uint32_t v) { return __builtin_bit_cast(u16x2, v); }
__device__ __forceinline__ uint32_t as_u32(u16x2 v) { return __builtin_bit_cast(uint32_t, v); }

// ---------------------------------------------------------------------------
// top-k lists: k u64 slots per trace, ascending, UINT64_MAX = empty
// ---------------------------------------------------------------------------
__device__ __forceinline__ void knn_insert(uint64_t *list, uint32_t k, uint64_t key) {
    if (key >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    for (uint32_t s = 0; s < k; ++s) {
        const uint64_t old = atomicMin((unsigned long long *)&list[s], (unsigned long long)key);
        if (old == UINT64_MAX) return;
        key = old > key ? old : key;
    }
}

__device__ __forceinline__ uint64_t wave_min_u64(uint64_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        const uint64_t o = __shfl_xor(v, off, 64);
        v = o < v ? o : v;
    }
    return v;
}

// insert the wave's k best keys for one query trace (all lanes participate)
__device__ __forceinline__ void knn_insert_wave(uint64_t *list, uint32_t k, uint64_t key, uint32_t lane) {
    for (uint32_t r = 0; r < k; ++r) {
        const uint64_t best = wave_min_u64(key);
        if (best == UINT64_MAX) return;
        if (best >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        if (lane == (uint32_t)__builtin_amdgcn_readfirstlane(__ffsll(__ballot(key == best)) - 1))
            knn_insert(list, k, best);
        if (key == best) key = UINT64_MAX;
    }
}

// ---------------------------------------------------------------------------
// wave -> (query pair, candidate group) over the upper triangle of 64x64 blocks
//   block b (queries 64b..64b+63 = 32 query pairs) x groups g in [b, G)
//   waves in block b: 32*(G-b); inner order keeps one candidate group for
//   32 consecutive waves (8 workgroups) so the group's symbols are re-read
//   from the same L2.
// ---------------------------------------------------------------------------
__host__ __device__ inline uint64_t tri_prefix(uint64_t b, uint64_t G) { return 32 * (b * G - b * (b - 1) / 2); }

struct EdArgs {
    const uint16_t *qsym;       // query symbols, CSR order
    const uint64_t *qoff;       // [N+1]
    const uint16_t *csym;       // candidate symbols, [group][pos][64]
    const uint64_t *coff;       // [G] element offset of each group block
    const uint32_t *gmax;       // [G] padded length of each group
    const uint32_t *len;        // [N]
    uint32_t N, G, k;
    uint64_t n_waves;           // waves of this shard
    uint32_t shard, n_shards;   // 32-wave groups dealt round-robin over shards
    uint64_t *knn;              // [N][k]
};

template <int W>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2))) void k_ed_tile(EdArgs A) {
    // at least two waves per SIMD: at W = 32 the compiler's own allocation was 256 VGPRs + 26 AGPRs (one wave); bound
    // to 256 it spills ~23 VGPRs (the row-block size R = 2, 4, 8 changes nothing)
    constexpr int R = ED_R;
    constexpr int NB = 2 * W + 1;       // band cells
    constexpr int NW = 2 * W + R;       // window symbols
    // XCD-aware: hardware block b runs on XCD b%8; give each XCD a contiguous
    // range of logical blocks so waves sharing a candidate group share an L2.
    const uint32_t nblk = gridDim.x, per_xcd = nblk / 8;
    const uint32_t hb = blockIdx.x;
    const uint32_t lb = (hb % 8) * per_xcd + hb / 8;
    const uint64_t lwave = (uint64_t)lb * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (lwave >= A.n_waves) return;
    const uint64_t wave = ((lwave / 32) * A.n_shards + A.shard) * 32 + lwave % 32;

    // locate block b: largest b with tri_prefix(b) <= wave
    uint32_t lo = 0, hi = A.G;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (tri_prefix(mid, A.G) <= wave) lo = mid; else hi = mid;
    }
    const uint32_t b = lo;
    const uint64_t idx = wave - tri_prefix(b, A.G);
    const uint32_t g = b + (uint32_t)(idx / 32);
    const uint32_t q1 = 64 * b + 2 * (uint32_t)(idx % 32), q2 = q1 + 1;
    const uint32_t j = 64 * g + lane;

    const bool v1 = q1 < A.N && j < A.N && j > q1;
    const bool v2 = q2 < A.N && j < A.N && j > q2;
    const uint32_t n1 = q1 < A.N ? A.len[q1] : 0, n2 = q2 < A.N ? A.len[q2] : 0;
    const uint32_t m = j < A.N ? A.len[j] : 0;
    const uint16_t *__restrict__ a1 = A.qsym + (q1 < A.N ? A.qoff[q1] : 0);
    const uint16_t *__restrict__ a2 = A.qsym + (q2 < A.N ? A.qoff[q2] : 0);
    const uint16_t *__restrict__ cs = A.csym + A.coff[g] + lane;
    const uint32_t glen = A.gmax[g];

    // per-half state: result, whether still running
    uint32_t r1 = W + 1, r2 = W + 1;
    bool run1 = v1, run2 = v2;
    const int32_t d1 = (int32_t)m - (int32_t)n1, d2 = (int32_t)m - (int32_t)n2;
    if (run1 && (d1 > W || d1 < -W)) run1 = false;  // |n-m| > W: W+1
    if (run2 && (d2 > W || d2 < -W)) run2 = false;
    if (run1 && n1 == 0) { r1 = m; run1 = false; }
    if (run2 && n2 == 0) { r2 = m; run2 = false; }

    const uint32_t nrows = __builtin_amdgcn_readfirstlane(max(n1, n2));  // n_h = 0 for q_h >= N
    u16x2 D[NB];
    uint32_t win[NW];  // packed (b, b) symbols for window positions i0-W .. i0-W+NW-1
#pragma unroll
    for (int t = 0; t < NB; ++t) D[t] = splat(t >= W ? (uint16_t)(t - W) : INF16);
    auto load_sym = [&](int64_t pos) -> uint32_t {
        const uint32_t s = (pos >= 0 && pos < (int64_t)glen) ? (uint32_t)cs[(uint64_t)pos * 64] : (uint32_t)CAND_PAD;
        return s | (s << 16);
    };
#pragma unroll
    for (int t = 0; t < NW; ++t) win[t] = load_sym((int64_t)t - W);

    const u16x2 one = splat(1);
    uint32_t i0 = 0;
    const bool any_run = __builtin_amdgcn_readfirstlane((uint32_t)__any(run1 || run2)) != 0;
    if (any_run) {
        while (i0 < nrows) {
            // next extraction row for the halves that are still alive
            const uint32_t stop = min(nrows, min(n1 > i0 ? n1 : nrows, n2 > i0 ? n2 : nrows));
            const uint32_t stop_u = __builtin_amdgcn_readfirstlane(stop);
            if (i0 + R <= stop_u) {
                // prefetch the symbols entering the window after this block
                uint32_t nxt[R];
#pragma unroll
                for (int r = 0; r < R; ++r) nxt[r] = load_sym((int64_t)i0 - W + NW + r);
#pragma unroll
                for (int r = 0; r < R; ++r) {
                    const uint32_t i = i0 + r;  // computing row i+1, symbols a[i]
                    const uint32_t s1 = i < n1 ? a1[i] : QUERY_PAD, s2 = i < n2 ? a2[i] : QUERY_PAD;
                    const uint32_t ap = __builtin_amdgcn_readfirstlane(s1 | (s2 << 16));
                    u16x2 left = splat(INF16);
#pragma unroll
                    for (int t = 0; t < NB; ++t) {
                        const u16x2 c = pk_min(as_pk(win[r + t] ^ ap), one);
                        const u16x2 diag = D[t] + c;
                        const u16x2 up = (t + 1 < NB) ? D[t + 1] : splat(INF16);
                        const u16x2 nd = pk_min(diag, pk_min(up, left) + one);
                        D[t] = nd;
                        left = nd;
                    }
                }
#pragma unroll
                for (int t = 0; t < NW - R; ++t) win[t] = win[t + R];
#pragma unroll
                for (int r = 0; r < R; ++r) win[NW - R + r] = nxt[r];
                i0 += R;
            } else {
                // single row (lands exactly on an extraction row)
                const uint32_t i = i0;
                const uint32_t s1 = i < n1 ? a1[i] : QUERY_PAD, s2 = i < n2 ? a2[i] : QUERY_PAD;
                const uint32_t ap = __builtin_amdgcn_readfirstlane(s1 | (s2 << 16));
                u16x2 left = splat(INF16);
#pragma unroll
                for (int t = 0; t < NB; ++t) {
                    const u16x2 c = pk_min(as_pk(win[t] ^ ap), one);
                    const u16x2 diag = D[t] + c;
                    const u16x2 up = (t + 1 < NB) ? D[t + 1] : splat(INF16);
                    const u16x2 nd = pk_min(diag, pk_min(up, left) + one);
                    D[t] = nd;
                    left = nd;
                }
                const uint32_t nx = load_sym((int64_t)i0 - W + NW);
#pragma unroll
                for (int t = 0; t < NW - 1; ++t) win[t] = win[t + 1];
                win[NW - 1] = nx;
                i0 += 1;
            }
            // extraction at row n_h: D(n, m) sits on diagonal m - n
            if (i0 == n1 && run1) {
                uint32_t v = W + 1;
#pragma unroll
                for (int t = 0; t < NB; ++t) v = (t - W == d1) ? (uint32_t)D[t].x : v;
                r1 = min(v, (uint32_t)W + 1);
                run1 = false;
            }
            if (i0 == n2 && run2) {
                uint32_t v = W + 1;
#pragma unroll
                for (int t = 0; t < NB; ++t) v = (t - W == d2) ? (uint32_t)D[t].y : v;
                r2 = min(v, (uint32_t)W + 1);
                run2 = false;
            }
            // cut-off: row band minimum > W stays > W
            if ((i0 & 15) == 0 || !(run1 || run2)) {
                u16x2 mn = D[0];
#pragma unroll
                for (int t = 1; t < NB; ++t) mn = pk_min(mn, D[t]);
                if (mn.x > W) run1 = false;
                if (mn.y > W) run2 = false;
                if (!__any(run1 || run2)) break;
            }
        }
    }
    // publish: candidate lists (per lane) and query lists (wave-reduced)
    const uint64_t key1 = v1 ? (((uint64_t)r1 << 32) | j) : UINT64_MAX;
    const uint64_t key2 = v2 ? (((uint64_t)r2 << 32) | j) : UINT64_MAX;
    if (v1) knn_insert(A.knn + (uint64_t)j * A.k, A.k, ((uint64_t)r1 << 32) | q1);
    if (v2) knn_insert(A.knn + (uint64_t)j * A.k, A.k, ((uint64_t)r2 << 32) | q2);
    if (q1 < A.N) knn_insert_wave(A.knn + (uint64_t)q1 * A.k, A.k, key1, lane);
    if (q2 < A.N) knn_insert_wave(A.knn + (uint64_t)q2 * A.k, A.k, key2, lane);
}

// ---------------------------------------------------------------------------
// generic: one thread per pair, u64 symbols, band row in global scratch
// ---------------------------------------------------------------------------
// ED_W(a, b) with the band row D[t] = cell (i, i + t - W) in global scratch (column t at scratch[t * stride]):
// one thread per pair, any band, any symbol type
template <typename T>
__device__ uint32_t generic_band_dist(const T *__restrict__ a, int64_t n, const T *__restrict__ b, int64_t m, uint32_t W,
                                      uint32_t *__restrict__ scratch, uint64_t stride) {
    const uint32_t NB = 2 * W + 1;
    const uint32_t INF = 0x3fffffffu;
    const int64_t dd = m - n;
    if (dd > (int64_t)W || dd < -(int64_t)W) return W + 1;
    // row 0: D(0, j) = j
    for (uint32_t t = 0; t < NB; ++t) scratch[t * stride] = (t >= W) ? (t - W) : INF;
    for (int64_t i = 1; i <= n; ++i) {
        uint32_t left = INF;
        for (uint32_t t = 0; t < NB; ++t) {
            const int64_t jj = i + (int64_t)t - (int64_t)W;
            uint32_t v;
            if (jj < 0 || jj > m) {
                v = INF;
            } else if (jj == 0) {
                v = (uint32_t)i;
            } else {
                const uint32_t diag = scratch[t * stride];
                const uint32_t up = (t + 1 < NB) ? scratch[(t + 1) * stride] : INF;
                v = diag + (a[i - 1] != b[jj - 1] ? 1u : 0u);
                v = min(v, min(up, left) + 1);
                v = min(v, INF);
            }
            scratch[t * stride] = v;
            left = v;
        }
    }
    return min(scratch[(uint32_t)(dd + W) * stride], W + 1);
}

__global__ __launch_bounds__(256) void k_ed_generic(const uint64_t *__restrict__ off, const uint64_t *__restrict__ sym,
                                                    const uint32_t *__restrict__ pairs, uint64_t n_pairs, uint32_t W,
                                                    uint32_t *__restrict__ scratch, uint32_t *__restrict__ dist) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t p = tid; p < n_pairs; p += nthr) {
        const uint32_t ia = pairs[2 * p], ib = pairs[2 * p + 1];
        dist[p] = generic_band_dist(sym + off[ia], (int64_t)(off[ia + 1] - off[ia]), sym + off[ib],
                                    (int64_t)(off[ib + 1] - off[ib]), W, scratch + tid, nthr);
    }
}

__device__ __forceinline__ void knn_insert_key(uint64_t *list, uint32_t k, uint64_t key) {
    if (key >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    for (uint32_t s = 0; s < k; ++s) {
        const uint64_t old = atomicMin((unsigned long long *)&list[s], (unsigned long long)key);
        if (old == UINT64_MAX) return;
        key = old > key ? old : key;
    }
}

// Single queries against a resident store without a bit-parallel query kernel (k_ed_tile's dense ids, the generic
// plan's u64 symbols, or a bit-parallel plan's encoded streams when a query pair's symbols overflow the compact
// tables): thread per (query, stored trace) pair; stored trace j at sym[soff[j]], length slen[j] (or the CSR
// difference when slen is NULL); in-band results into the query's list
__global__ __launch_bounds__(256) void k_ed_query_generic(const uint64_t *__restrict__ soff,
                                                          const uint32_t *__restrict__ slen, const void *__restrict__ sym,
                                                          bool wide_sym, const uint64_t *__restrict__ qstart,
                                                          const uint32_t *__restrict__ qlen, const void *__restrict__ qsym,
                                                          uint32_t n_q, uint32_t N, uint32_t W, uint32_t k,
                                                          uint32_t *__restrict__ scratch, uint64_t *__restrict__ knn) {
    const uint64_t nthr = (uint64_t)gridDim.x * blockDim.x;
    const uint64_t tid = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    for (uint64_t p = tid; p < (uint64_t)n_q * N; p += nthr) {
        const uint32_t q = (uint32_t)(p / N), j = (uint32_t)(p % N);
        const int64_t n = qlen[q], m = slen ? (int64_t)slen[j] : (int64_t)(soff[j + 1] - soff[j]);
        const uint32_t r = wide_sym
            ? generic_band_dist((const uint64_t *)qsym + qstart[q], n, (const uint64_t *)sym + soff[j], m, W,
                                scratch + tid, nthr)
            : generic_band_dist((const uint16_t *)qsym + qstart[q], n, (const uint16_t *)sym + soff[j], m, W,
                                scratch + tid, nthr);
        if (r <= W) knn_insert_key(knn + (uint64_t)q * k, k, ((uint64_t)r << 32) | j);
    }
}

__global__ void k_knn_init(uint64_t *knn, uint64_t n) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) knn[i] = UINT64_MAX;
}

// a search's start: its k-NN lists and (bit-parallel plans) the work counters in one launch (a separate memset of
// the counters was one more queue entry per search, ~5 us: a shard of a sharded search pays it once per shard)
__global__ void k_knn_init_cnt(uint64_t *knn, uint64_t n, uint64_t *counters, uint32_t n_cnt) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) knn[i] = UINT64_MAX;
    if (counters && i < n_cnt) counters[i] = 0;
}

__global__ void k_knn_final(const uint64_t *__restrict__ knn, uint64_t n, uint32_t *__restrict__ ids,
                            uint32_t *__restrict__ ds) {
    uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint64_t key = knn[i];
    ids[i] = key == UINT64_MAX ? NMZ_NONE : (uint32_t)key;
    ds[i] = key == UINT64_MAX ? NMZ_NONE : (uint32_t)(key >> 32);
}

// Complete k-NN lists whose listed keys are the results within the band (dist < fill_d): every pair not listed has
// the result fill_d = band + 1, so list i takes (fill_d, j) for the smallest ids j < n_cand not listed (j != i when
// self_exclude), in increasing j, until it holds k keys (UINT64_MAX where fewer candidates exist). Keys at or
// above fill_d already in the list (kernels that list every pair) are recomputed to the same values.
__global__ void k_knn_fill(uint64_t *knn, uint32_t n_lists, uint32_t k, uint32_t n_cand, uint32_t fill_d,
                           int self_exclude) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n_lists) return;
    uint64_t *L = knn + (uint64_t)i * k;
    uint32_t c = 0;
    while (c < k && L[c] != UINT64_MAX && (uint32_t)(L[c] >> 32) < fill_d) ++c;
    uint32_t j = 0;
    for (uint32_t s = c; s < k; ++s) {
        for (;; ++j) {
            if (j >= n_cand) break;
            if (self_exclude && j == i) continue;
            bool listed = false;
            for (uint32_t t = 0; t < c; ++t) listed |= (uint32_t)L[t] == j;
            if (!listed) break;
        }
        L[s] = j < n_cand ? (((uint64_t)fill_d << 32) | j) : UINT64_MAX;
        ++j;
    }
}

// all-pairs via the generic kernel (fallback): pair list = upper triangle
__global__ void k_pairs_upper(uint32_t N, uint64_t start, uint64_t count, uint32_t *pairs) {
    uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    uint64_t p = start + t;  // p-th pair (i<j), row-major
    // i = largest with i*(2N-i-1)/2 <= p
    double Nd = N;
    uint64_t i = (uint64_t)floor(((2 * Nd - 1) - sqrt((2 * Nd - 1) * (2 * Nd - 1) - 8.0 * (double)p)) / 2);
    auto base = [&](uint64_t r) { return r * (2 * (uint64_t)N - r - 1) / 2; };
    while (i > 0 && base(i) > p) --i;
    while (base(i + 1) <= p) ++i;
    const uint64_t jj = i + 1 + (p - base(i));
    pairs[2 * t] = (uint32_t)i;
    pairs[2 * t + 1] = (uint32_t)jj;
}

__global__ void k_knn_from_pairs(const uint32_t *__restrict__ pairs, const uint32_t *__restrict__ dist, uint64_t count,
                                 uint64_t *knn, uint32_t k) {
    uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (t >= count) return;
    const uint32_t i = pairs[2 * t], j = pairs[2 * t + 1];
    const uint64_t d = dist[t];
    knn_insert(knn + (uint64_t)i * k, k, (d << 32) | j);
    knn_insert(knn + (uint64_t)j * k, k, (d << 32) | i);
}

}  // namespace nmz

// ---------------------------------------------------------------------------
// ED plan: symbol remap + device layouts (reused across searches)
// ---------------------------------------------------------------------------
struct nmz_ed_plan {
    nmz_ctx *ctx = nullptr;
    uint32_t n = 0, band = 0, G = 0;
    bool fast = false;
    bool bv = false;               // bit-parallel kernel (k_ed_bv) usable
    uint64_t *d_soff = nullptr;    // bv: per-trace stream offsets
    uint32_t pool = 0;
    bool wide = false;             // wide-band bit-parallel kernel (k_ed_wide) usable
    bool tile = false;             // k_ed_tile (dense ids in d_qsym / d_qoff)
    uint32_t n_sym = 0;
    uint32_t *d_peq = nullptr;     // wide: [N][n_sym][ndw] match bitmaps
    uint32_t *d_rowb = nullptr;    // wide: per-position Peq row byte offsets (EdWideArgs::rowb)
    uint64_t *d_rowb_off = nullptr;
    uint32_t ndw = 0, lds_dw = 0;  // bv: dwords per Peq row per query, LDS dwords per workgroup
    uint64_t n_chunks = 0;         // bv: total chunks (64-query block row x ED_BV_POOL candidates)
    uint16_t *d_bsym = nullptr;
    uint64_t *d_chunk_start = nullptr;  // bv: [G+1] per-row chunk starts (single-kernel search)
    std::vector<uint64_t> row_chunks;    // bv: chunks per block row
    uint64_t *d_counters = nullptr;  // bv: work counters of the latest search (nmz_ed_plan_counters)
    uint32_t *d_prof = nullptr;      // bv: [N][ED_QG_DW] q-gram profiles (ed_qgram_profiles)
    uint32_t rq = 64;                // bv: queries per block row
    uint32_t maxlen = 0;
    uint32_t bw = 0;                 // bv: the kernels' template band W >= band (8, 16, 32, 64)
    bool cmp = false;                // bv: compact tables (streams of symbol ids, per-workgroup rows; ed_bv.hip)
    uint32_t rmap_dw = 0, claim_dw = 0, row_bytes = 0;  // bv, compact: LDS layout (EdBvArgs)
    uint32_t ww = 0;                 // wide: the kernel's W (1024 * 2^k >= band)
    std::unordered_map<uint64_t, uint32_t> dict;  // bv: symbol -> dense id (single-query search)
    nmz::DevBuf mem;
    // bv, two-phase search: per-(shard, n_shards) tile starts (host, kept), scratch and the entry lists
    std::map<uint64_t, nmz::DevBuf> tile_list;      // per (shard, n_shards): the shard's tiles (qb << 32 | cb)
    std::map<uint64_t, uint64_t> tile_count;
    nmz::DevBuf tp_mem, tp_ent, tp_rec;
    struct TpSizes {
        uint64_t tot64;
        uint32_t items, n_rec, item;
    };
    std::map<uint64_t, TpSizes> tp_sizes;  // per (shard, n_shards): entry total, DP items, records of its searches
    uint32_t *d_tp_mismatch = nullptr;     // (in tp_mem) set when a search's totals differ from tp_sizes
    uint64_t tp_mem_gen = 0, tp_rec_gen = 0;  // DevBuf::gen of tp_mem / tp_rec when their counters were last cleared
    bool tp_dirty = false;                 // a count pass's counts not yet taken back by its write pass
    // the mismatch flag as of the last search enqueued with cached sizes: that search's offsets scan writes {its
    // sequence number, the flag} to these pinned words, read (ed_tp_flag_check) by the shard's next search without
    // waiting once the number has landed, or read from the device with a wait by the synchronous entry points
    // (nmz_ed_plan_counters, the group search)
    uint32_t *h_tp_flag = nullptr;
    uint32_t tp_seq = 0;       // the latest cached search's number
    uint32_t tp_seq_sent = 0;  // the latest number whose scan was enqueued (the last writer of h_tp_flag)
    bool tp_flag_armed = false;
    // fixed at creation (NMZ_ED_QGRAM / NMZ_ED_TWO_PHASE, A/B knobs read once per plan), so every shard and every
    // call of one plan takes the same search and deals pairs by the same rule
    bool qgram = true, two_phase = true;
    uint32_t opts = 0;               // NMZ_ED_OPT_* the plan was created with (options | A/B knobs)
    uint64_t total = 0, off_hash = 0;  // symbols in the store; FNV-1a of its offsets (nmz_ed_plan_fingerprint)
    uint16_t *d_qsym = nullptr, *d_csym = nullptr;
    uint64_t *d_qoff = nullptr, *d_coff = nullptr;
    uint32_t *d_gmax = nullptr, *d_len = nullptr;
    // generic path
    uint64_t *d_off64 = nullptr, *d_sym64 = nullptr;
};

namespace nmz {

// stored streams of the bit-parallel plan from device symbols: one block per trace, each symbol's dense id is its
// rank among the sorted distinct symbols (binary search), written as its Peq row's byte offset (id * ndw * 8), or
// as the id itself for compact tables (row_bytes = 1)
__global__ __launch_bounds__(256) void k_ed_bv_remap(const uint64_t *__restrict__ off, const uint64_t *__restrict__ sym,
                                                     const uint64_t *__restrict__ uniq, uint32_t n_uniq,
                                                     const uint64_t *__restrict__ soff, uint32_t row_bytes,
                                                     uint16_t *__restrict__ bs) {
    const uint32_t i = blockIdx.x;
    const uint64_t b = off[i], n = off[i + 1] - b, so = soff[i];
    for (uint64_t t = threadIdx.x; t < n; t += 256) {
        const uint64_t x = sym[b + t];
        uint32_t lo = 0, hi = n_uniq;  // first index with uniq[idx] >= x (x is present)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (uniq[mid] < x) lo = mid + 1; else hi = mid;
        }
        bs[so + t] = (uint16_t)(lo * row_bytes);
    }
}

// per trace: the number of distinct stream values (symbol ids < n_ids), one workgroup per trace with an LDS bitmap
__global__ __launch_bounds__(256) void k_trace_distinct(const uint16_t *__restrict__ bs, const uint64_t *__restrict__ soff,
                                                        const uint32_t *__restrict__ len, uint32_t n_ids,
                                                        uint32_t *__restrict__ out) {
    extern __shared__ uint32_t bits[];
    const uint32_t i = blockIdx.x, nw = (n_ids + 31) / 32;
    for (uint32_t t = threadIdx.x; t < nw; t += 256) bits[t] = 0;
    __syncthreads();
    const uint16_t *a = bs + soff[i];
    for (uint32_t t = threadIdx.x; t < len[i]; t += 256) atomicOr(&bits[a[t] >> 5], 1u << (a[t] & 31));
    __syncthreads();
    uint32_t c = 0;
    for (uint32_t t = threadIdx.x; t < nw; t += 256) c += __builtin_popcount(bits[t]);
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) c += __shfl_xor(c, off, 64);
    __shared__ uint32_t part[4];
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) out[i] = part[0] + part[1] + part[2] + part[3];
}

// LDS extras of the pool kernels beyond the tables: counters, two q-gram profiles, a pool's survivor list
static size_t bv_pool_extras(uint32_t pool) { return 16 + 2 * ED_QG_DW * 4 + ((size_t)pool * 2 + 15) / 16 * 16; }

// Compact bit-parallel tables (ed_bv.hip CMP): R rows for a workgroup's queries + the zero row, the map of
// n_ids symbol ids (+ the padding id) to row byte offsets (u16), the claim bitmap. False when they do not fit
// `limit` bytes with `extras` (or a row offset would not fit 16 bits).
static bool bv_compact_layout(uint32_t n_ids, uint32_t R, uint32_t ndw, size_t extras, size_t limit, uint32_t &lds_dw,
                              uint32_t &rmap_dw, uint32_t &claim_dw) {
    const uint64_t rows_bytes = (uint64_t)(R + 1) * ndw * 8;
    const uint64_t peq_dw = (rows_bytes / 4 + 3) / 4 * 4;
    const uint64_t map_dw = ((n_ids + 2) / 2 + 3) / 4 * 4;
    const uint64_t clm_dw = ((n_ids + 32) / 32 + 3) / 4 * 4;
    const uint64_t total = peq_dw + map_dw + clm_dw;
    if (rows_bytes > 65535 || total * 4 + extras > limit) return false;
    lds_dw = (uint32_t)total;
    rmap_dw = (uint32_t)peq_dw;
    claim_dw = (uint32_t)(peq_dw + map_dw);
    return true;
}

// the largest d(2p) + d(2p + 1) over the query pairs (the rows one workgroup's compact tables need)
static uint32_t pair_rows_max(const std::vector<uint32_t> &d) {
    uint32_t r = 0;
    for (size_t i = 0; i < d.size(); i += 2) r = std::max(r, d[i] + (i + 1 < d.size() ? d[i + 1] : 0u));
    return r;
}

constexpr uint64_t ED_DEVICE_REMAP_MIN = 1ULL << 20;

// the q-gram lower-bound filter of the bit-parallel kernels (ed_bv.hip); NMZ_ED_QGRAM=0 turns it off for A/B runs
// the two-phase search (filter tiles, then DP work items) when the q-gram filter is on; NMZ_ED_TWO_PHASE=0 keeps
// the single-kernel search with its in-workgroup pre-filter (A/B runs)
static bool ed_two_phase_enabled() {
    const char *e = ab_env("NMZ_ED_TWO_PHASE");
    return !(e && atoi(e) == 0);
}

static bool ed_qgram_enabled() {
    const char *e = ab_env("NMZ_ED_QGRAM");
    return !(e && atoi(e) == 0);
}

// queries per block row of the bit-parallel search (NMZ_ED_RW overrides the multiple of 64 for A/B runs)
static uint32_t ed_bv_row_queries() {
    static const uint32_t rq = [] {
        const char *e = ab_env("NMZ_ED_RW");
        const int v = e ? atoi(e) : (int)ED_BV_RW;
        return 64u * (uint32_t)((v >= 1 && v <= 32) ? v : (int)ED_BV_RW);
    }();
    return rq;
}  // symbols; smaller stores keep the host remap

// The bit-parallel plan built on the device: upload the symbols, sort/unique them (dense ids = ranks), write the
// candidate streams with a binary search per symbol. Returns 1 (not applicable: the alphabet does not fit the
// bit-parallel LDS tables) so the caller falls back to the host build and the other kernels.
// d_sym_in: the symbols already on the device (nmz_ed_plan_create_dev), else uploaded from sym.
static int ed_plan_build_bv_device(nmz_ed_plan *p, const uint64_t *off, const uint64_t *sym, uint32_t N,
                                   uint32_t band, uint32_t maxlen, const uint64_t *d_sym_in, bool compact_opt) {
    hipStream_t st = p->ctx->stream;
    const uint64_t total = off[N];
    NMZ_CHECK(total == 0 || sym || d_sym_in, "sym is NULL");
    DevBuf tmp;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } release_tmp{tmp};
    NMZ_TRY(tmp.ensure(Carve::bytes_for(d_sym_in ? 0 : total, 8) + Carve::bytes_for(MAX_FAST_SYMBOLS + 1, 8) +
                       Carve::bytes_for(N + 1, 8)));
    Carve tv(tmp.ptr);
    const uint64_t *d_sym = d_sym_in;
    if (!d_sym_in) {
        uint64_t *d_up = tv.take<uint64_t>(total);
        NMZ_HIP(hipMemcpyAsync(d_up, sym, total * 8, hipMemcpyHostToDevice, st));
        d_sym = d_up;
    }
    uint64_t *d_uniq = tv.take<uint64_t>(MAX_FAST_SYMBOLS + 1);
    uint64_t *d_off = tv.take<uint64_t>(N + 1);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (N + 1) * 8, hipMemcpyHostToDevice, st));
    uint64_t n_uniq = 0;
    NMZ_TRY(device_unique_u64(d_sym, total, d_uniq, MAX_FAST_SYMBOLS, &n_uniq, st));
    const uint32_t bw = ed_bv_template(band);
    const uint32_t KF = (2 * bw + 31) / 32;
    const uint32_t ndw = ((maxlen + 31) / 32 + KF + 2) | 1;
    if (n_uniq >= MAX_FAST_SYMBOLS) return 1;
    const uint32_t rq = ed_bv_row_queries();
    const uint32_t n_sym = (uint32_t)n_uniq, G = (N + rq - 1) / rq;
    p->pool = N >= 24576 ? 4 * ED_BV_POOL : (N >= 12288 ? 2 * ED_BV_POOL : ED_BV_POOL);
    if (const char *e = ab_env("NMZ_ED_POOL")) {
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= 256 && v % 256 == 0 && v <= 16384) p->pool = v;
    }
    // direct tables (every symbol of the store has a row) when they fit beside the pool kernels' extras, else
    // compact tables (decided after the streams exist: they need the traces' distinct counts)
    const uint64_t direct_bytes = (((uint64_t)(n_sym + 1) * ndw * 8 + 15) / 16) * 16;
    const bool cmp = direct_bytes + bv_pool_extras(p->pool) > 65536 || compact_opt;
    if (cmp) p->pool = std::min(p->pool, ED_BV_POOL);  // the single kernel's survivor list leaves room for rows
    p->bv = true;
    p->fast = true;
    p->bw = bw;
    p->cmp = cmp;
    p->ndw = ndw;
    p->row_bytes = ndw * 8;
    p->lds_dw = (uint32_t)(direct_bytes / 4);
    p->G = G;
    p->rq = rq;
    p->maxlen = maxlen;
    p->n_sym = n_sym;
    // padding value: the zero row's offset (direct), or the id n_sym, which no workgroup ever gives a row (compact)
    const uint32_t zero_row = cmp ? n_sym : n_sym * ndw * 8;
    std::vector<uint32_t> len(N + 1, 0);
    std::vector<uint64_t> soff(N + 1, 0), chunk_start(G + 1, 0);
    for (uint32_t i = 0; i < N; ++i) {
        len[i] = (uint32_t)(off[i + 1] - off[i]);
        soff[i + 1] = soff[i] + ((uint64_t)(len[i] + 31) / 32 + 1) * 32;
    }
    for (uint32_t b = 0; b < G; ++b) chunk_start[b + 1] = chunk_start[b] + (N - rq * b + p->pool - 1) / p->pool;
    p->n_chunks = chunk_start[G];
    p->row_chunks.resize(G);
    for (uint32_t b = 0; b < G; ++b) p->row_chunks[b] = chunk_start[b + 1] - chunk_start[b];
    const uint64_t bs_n = soff[N] + 64;
    NMZ_TRY(p->mem.ensure(Carve::bytes_for(bs_n, 2) + Carve::bytes_for(N + 1, 8) * 2 + Carve::bytes_for(G + 1, 8) +
                          Carve::bytes_for(N + 1, 4) + Carve::bytes_for(ED_CNT_WORDS, 8) +
                          Carve::bytes_for((uint64_t)N * ED_QG_DW, 4)));
    Carve cv(p->mem.ptr);
    p->d_counters = cv.take<uint64_t>(ED_CNT_WORDS);
    p->d_prof = cv.take<uint32_t>((uint64_t)N * ED_QG_DW);
    p->d_bsym = cv.take<uint16_t>(bs_n);
    p->d_soff = cv.take<uint64_t>(N + 1);
    p->d_qoff = cv.take<uint64_t>(N + 1);
    p->d_chunk_start = cv.take<uint64_t>(G + 1);
    p->d_len = cv.take<uint32_t>(N + 1);
    NMZ_HIP(hipMemsetD16Async((hipDeviceptr_t)p->d_bsym, (unsigned short)zero_row, bs_n, st));
    NMZ_HIP(hipMemcpyAsync(p->d_soff, soff.data(), (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(p->d_qoff, off, (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(p->d_chunk_start, chunk_start.data(), (G + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(p->d_len, len.data(), (N + 1) * 4, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemsetAsync(p->d_counters, 0, ED_CNT_WORDS * 8, st));
    hipLaunchKernelGGL(k_ed_bv_remap, dim3(N), dim3(256), 0, st, d_off, d_sym, d_uniq, n_sym, p->d_soff,
                       cmp ? 1u : ndw * 8, p->d_bsym);
    NMZ_HIP(hipGetLastError());
    if (cmp) {  // the traces' distinct counts size the per-workgroup rows
        DevBuf dbuf;
        struct R2 {
            DevBuf &b;
            ~R2() { b.release(); }
        } rel{dbuf};
        NMZ_TRY(dbuf.ensure(Carve::bytes_for(N + 1, 4)));
        hipLaunchKernelGGL(k_trace_distinct, dim3(N), dim3(256), ((n_sym + 32) / 32) * 4, st, p->d_bsym, p->d_soff,
                           p->d_len, n_sym + 1, dbuf.as<uint32_t>());
        NMZ_HIP(hipGetLastError());
        std::vector<uint32_t> d(N);
        NMZ_HIP(hipMemcpyAsync(d.data(), dbuf.ptr, (uint64_t)N * 4, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        if (!bv_compact_layout(n_sym, pair_rows_max(d), ndw, bv_pool_extras(p->pool), 65536, p->lds_dw, p->rmap_dw,
                               p->claim_dw))
            return 1;  // even a query pair's own symbols do not fit: the host build's other kernels
    }
    NMZ_TRY(ed_qgram_profiles(p->d_bsym, p->d_soff, p->d_len, N, p->d_prof, st));
    // the dictionary for single queries (nmz_ed_plan_query_knn): symbol -> rank
    std::vector<uint64_t> uniq(n_sym);
    NMZ_HIP(hipMemcpyAsync(uniq.data(), d_uniq, (uint64_t)n_sym * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    p->dict.reserve(n_sym * 2);
    for (uint32_t i = 0; i < n_sym; ++i) p->dict.emplace(uniq[i], i);
    return NMZ_OK;
}

// wide-band plan streams from device symbols: dense id (rank among the sorted distinct symbols) per position, in
// CSR order (qsym), and the id's Peq row byte offset per position of each trace's padded row stream (rowb)
__global__ __launch_bounds__(256) void k_ed_wide_remap(const uint64_t *__restrict__ off, const uint64_t *__restrict__ sym,
                                                       const uint64_t *__restrict__ uniq, uint32_t n_uniq,
                                                       const uint64_t *__restrict__ roff, uint32_t row_bytes,
                                                       uint16_t *__restrict__ qsym, uint32_t *__restrict__ rowb) {
    const uint32_t i = blockIdx.x;
    const uint64_t b = off[i], n = off[i + 1] - b, ro = roff[i];
    for (uint64_t t = threadIdx.x; t < n; t += 256) {
        const uint64_t x = sym[b + t];
        uint32_t lo = 0, hi = n_uniq;  // first index with uniq[idx] >= x (x is present)
        while (lo < hi) {
            const uint32_t mid = (lo + hi) >> 1;
            if (uniq[mid] < x) lo = mid + 1; else hi = mid;
        }
        qsym[b + t] = (uint16_t)lo;
        rowb[ro + t] = lo * row_bytes;
    }
}

// The wide-band plan built on the device (the host build remaps every symbol through a hash map: ~100 ms for
// configs[4]'s 1.7e7 symbols): distinct symbols from the device hash set, then one remap kernel. Returns 1 (not
// applicable: alphabet or Peq tables too large) so the caller takes the host build.
static int ed_plan_build_wide_device(nmz_ed_plan *p, const uint64_t *off, const uint64_t *sym, uint32_t N,
                                     uint32_t band, uint32_t maxlen, const uint64_t *d_sym_in) {
    hipStream_t st = p->ctx->stream;
    const uint64_t total = off[N];
    NMZ_CHECK(total == 0 || sym || d_sym_in, "sym is NULL");
    DevBuf tmp;
    struct Release {
        DevBuf &b;
        ~Release() { b.release(); }
    } release_tmp{tmp};
    NMZ_TRY(tmp.ensure(Carve::bytes_for(d_sym_in ? 0 : total, 8) + Carve::bytes_for(MAX_FAST_SYMBOLS + 1, 8) +
                       Carve::bytes_for(N + 1, 8) * 2));
    Carve tv(tmp.ptr);
    const uint64_t *d_sym = d_sym_in;
    if (!d_sym_in) {
        uint64_t *d_up = tv.take<uint64_t>(total);
        NMZ_HIP(hipMemcpyAsync(d_up, sym, total * 8, hipMemcpyHostToDevice, st));
        d_sym = d_up;
    }
    uint64_t *d_uniq = tv.take<uint64_t>(MAX_FAST_SYMBOLS + 1);
    uint64_t *d_off = tv.take<uint64_t>(N + 1), *d_roff = tv.take<uint64_t>(N + 1);
    uint64_t n_uniq = 0;
    NMZ_TRY(device_unique_u64(d_sym, total, d_uniq, MAX_FAST_SYMBOLS, &n_uniq, st));
    if (n_uniq >= MAX_FAST_SYMBOLS) return 1;
    const uint32_t n_sym = std::max((uint32_t)n_uniq, 1u);
    p->ww = ed_wide_template(band);
    const uint32_t ndw = ed_wide_ndw(p->ww, maxlen);
    const uint64_t peq_bytes = (uint64_t)N * n_sym * ndw * 4;
    if (peq_bytes > (16ULL << 30) || (uint64_t)n_sym * ndw * 4 >= (1ULL << 31)) return 1;
    p->wide = true;
    p->fast = true;
    p->ndw = ndw;
    p->n_sym = n_sym;
    std::vector<uint64_t> roff(N + 1, 0);
    for (uint32_t i = 0; i < N; ++i) roff[i + 1] = roff[i] + ((off[i + 1] - off[i] + 31) / 32 + 2) * 32;
    const uint64_t nrow = roff[N] + 1;
    NMZ_TRY(p->mem.ensure(Carve::bytes_for(total + 64, 2) + Carve::bytes_for(N + 1, 8) +
                          Carve::bytes_for((uint64_t)N * n_sym * ndw, 4) + Carve::bytes_for(nrow, 4) +
                          Carve::bytes_for(N + 1, 8)));
    Carve cv(p->mem.ptr);
    p->d_qsym = cv.take<uint16_t>(total + 64);
    p->d_qoff = cv.take<uint64_t>(N + 1);
    p->d_peq = cv.take<uint32_t>((uint64_t)N * n_sym * ndw);
    p->d_rowb = cv.take<uint32_t>(nrow);
    p->d_rowb_off = cv.take<uint64_t>(N + 1);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_roff, roff.data(), (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(p->d_qoff, off, (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(p->d_rowb_off, roff.data(), (N + 1) * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemsetAsync(p->d_qsym, 0, (total + 64) * 2, st));
    NMZ_HIP(hipMemsetAsync(p->d_rowb, 0, nrow * 4, st));
    if (N) {
        hipLaunchKernelGGL(k_ed_wide_remap, dim3(N), dim3(256), 0, st, d_off, d_sym, d_uniq, (uint32_t)n_uniq, d_roff,
                           ndw * 4, p->d_qsym, p->d_rowb);
        NMZ_HIP(hipGetLastError());
    }
    NMZ_TRY(ed_wide_build_peq(p->d_qsym, p->d_qoff, N, n_sym, ndw, p->ww, p->d_peq, st));
    // the dictionary for single queries (nmz_ed_plan_query_knn): symbol -> rank
    std::vector<uint64_t> uniq(n_uniq);
    if (n_uniq) NMZ_HIP(hipMemcpyAsync(uniq.data(), d_uniq, n_uniq * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));  // the host vectors above are pageable; the scratch goes back
    p->dict.reserve(n_uniq * 2);
    for (uint64_t i = 0; i < n_uniq; ++i) p->dict.emplace(uniq[i], (uint32_t)i);
    p->maxlen = maxlen;
    return NMZ_OK;
}

// d_sym: the symbols on the device instead of sym (host); the host build paths take a copy of them
static int ed_plan_build(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t N, uint32_t band,
                         nmz_ed_plan **out, const uint64_t *d_sym = nullptr, uint32_t opts = 0) {
    NMZ_CHECK(ctx && out, "NULL argument");
    NMZ_CHECK(N == 0 || off, "off is NULL");
    NMZ_CHECK((opts & ~(uint32_t)(NMZ_ED_OPT_SINGLE_KERNEL | NMZ_ED_OPT_NO_QGRAM | NMZ_ED_OPT_COMPACT |
                                  NMZ_ED_OPT_HOST_BUILD)) == 0, "unknown plan option bits");
    // the A/B environment knobs (NMZ_AB=1 only) add to the options
    if (!ed_two_phase_enabled()) opts |= NMZ_ED_OPT_SINGLE_KERNEL;
    if (!ed_qgram_enabled()) opts |= NMZ_ED_OPT_NO_QGRAM;
    if (ab_env("NMZ_ED_COMPACT")) opts |= NMZ_ED_OPT_COMPACT;
    if (ab_env("NMZ_ED_HOST_REMAP")) opts |= NMZ_ED_OPT_HOST_BUILD;
    *out = nullptr;
    auto *p = new nmz_ed_plan();
    auto init = [&] {
        p->qgram = !(opts & NMZ_ED_OPT_NO_QGRAM);
        p->two_phase = !(opts & NMZ_ED_OPT_SINGLE_KERNEL);
        p->opts = opts;
        p->ctx = ctx;
        p->n = N;
        p->band = band;
        p->total = N ? off[N] : 0;
        uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a over the offsets: the store's shape, for the fingerprint
        for (uint32_t i = 0; i <= N; ++i) h = (h ^ off[i]) * 0x100000001b3ull;
        p->off_hash = h;
    };
    init();
    const bool compact_opt = (opts & NMZ_ED_OPT_COMPACT) != 0, host_build = (opts & NMZ_ED_OPT_HOST_BUILD) != 0;
    hipStream_t st = ctx->stream;
    const uint64_t total = N ? off[N] : 0;
    uint32_t maxlen = 0;
    for (uint32_t i = 0; i < N; ++i) maxlen = std::max<uint32_t>(maxlen, (uint32_t)(off[i + 1] - off[i]));
    if (ed_bv_supported(band) && maxlen + ed_bv_template(band) < MAX_FAST_LEN && total >= ED_DEVICE_REMAP_MIN &&
        total < (1ULL << 31) && !host_build) {
        const int rc = ed_plan_build_bv_device(p, off, sym, N, band, maxlen, d_sym, compact_opt);
        if (rc == NMZ_OK) {
            *out = p;
            return NMZ_OK;
        }
        p->mem.release();
        const bool not_applicable = rc == 1;
        delete p;
        if (!not_applicable) return rc;
        p = new nmz_ed_plan();  // alphabet too large for the bit-parallel tables: host build below
        init();
    }
    if (ed_wide_supported(band) && total >= ED_DEVICE_REMAP_MIN && !host_build) {
        const int rc = ed_plan_build_wide_device(p, off, sym, N, band, maxlen, d_sym);
        if (rc == NMZ_OK) {
            *out = p;
            return NMZ_OK;
        }
        p->mem.release();
        delete p;
        if (rc != 1) return rc;
        p = new nmz_ed_plan();  // alphabet or tables too large: the host build below
        init();
    }
    std::vector<uint64_t> hsym;  // the host paths read the symbols on the host
    if (d_sym && total) {
        hsym.resize(total);
        NMZ_HIP(hipMemcpyAsync(hsym.data(), d_sym, total * 8, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        sym = hsym.data();
    }
    NMZ_CHECK(total == 0 || sym, "sym is NULL");
    // dense symbol ids (exact remap: a == b <=> id(a) == id(b))
    std::vector<uint16_t> ids;
    const bool want_wide = ed_wide_supported(band);
    const bool want_bv = ed_bv_supported(band) && maxlen + ed_bv_template(band) < MAX_FAST_LEN;
    const bool tile_band = band == 8 || band == 16 || band == 32;  // k_ed_tile computes exactly its W
    bool fast = want_bv || want_wide;
    std::unordered_map<uint64_t, uint32_t> dict;
    if (fast) {
        dict.reserve(1024);
        ids.resize(total);
        for (uint64_t t = 0; t < total && fast; ++t) {
            auto it = dict.find(sym[t]);
            uint32_t id;
            if (it == dict.end()) {
                id = (uint32_t)dict.size();
                if (id >= MAX_FAST_SYMBOLS) fast = false;
                dict.emplace(sym[t], id);
            } else {
                id = it->second;
            }
            ids[t] = (uint16_t)id;
        }
    }
    auto cleanup = [&](int code) {
        p->mem.release();
        delete p;
        return code;
    };
    // bit-parallel path: per-query Peq rows for every symbol of the alphabet in LDS (direct tables), or for the
    // symbols of one query pair only (compact tables)
    uint32_t n_sym = 0;
    const uint32_t pool0 = [&] {
        uint32_t pl = N >= 24576 ? 4 * ED_BV_POOL : (N >= 12288 ? 2 * ED_BV_POOL : ED_BV_POOL);
        if (const char *e = ab_env("NMZ_ED_POOL")) {
            const uint32_t v = (uint32_t)atoi(e);
            if (v >= 256 && v % 256 == 0 && v <= 16384) pl = v;
        }
        return pl;
    }();
    if (fast && want_bv) {
        n_sym = (uint32_t)dict.size();
        const uint32_t bw = ed_bv_template(band);
        const uint32_t KF = (2 * bw + 31) / 32;
        uint32_t ndw = (maxlen + 31) / 32 + KF + 2;
        ndw |= 1;  // odd row stride: rows of distinct symbols start on distinct bank pairs
        const uint64_t lds_bytes = (((uint64_t)(n_sym + 1) * ndw * 8 + 15) / 16) * 16;
        p->bw = bw;
        p->ndw = ndw;
        p->row_bytes = ndw * 8;
        if (lds_bytes + bv_pool_extras(pool0) <= 65536 && !compact_opt) {
            p->bv = true;
            p->lds_dw = (uint32_t)(lds_bytes / 4);
        } else {
            std::vector<uint32_t> d(N, 0), stamp(n_sym + 1, UINT32_MAX);
            for (uint32_t i = 0; i < N; ++i)
                for (uint64_t t = off[i]; t < off[i + 1]; ++t)
                    if (stamp[ids[t]] != i) {
                        stamp[ids[t]] = i;
                        ++d[i];
                    }
            if (bv_compact_layout(n_sym, pair_rows_max(d), ndw, bv_pool_extras(std::min(pool0, ED_BV_POOL)), 65536,
                                  p->lds_dw, p->rmap_dw, p->claim_dw)) {
                p->bv = true;
                p->cmp = true;
            }
        }
    }
    if (fast && want_wide) {
        n_sym = (uint32_t)dict.size();
        p->ww = ed_wide_template(band);
        const uint32_t ndw = ed_wide_ndw(p->ww, maxlen);
        const uint64_t peq_bytes = (uint64_t)N * std::max(n_sym, 1u) * ndw * 4;
        // one query's table must be addressable by a 32-bit buffer offset
        if (peq_bytes <= (16ULL << 30) && (uint64_t)std::max(n_sym, 1u) * ndw * 4 < (1ULL << 31)) {
            p->wide = true;
            p->ndw = ndw;
            p->n_sym = std::max(n_sym, 1u);
        } else {
            fast = false;
        }
    }
    p->fast = fast;
    p->maxlen = maxlen;
    if (fast && p->wide) {
        // per-position Peq row byte offsets, each trace padded to whole 32-column blocks + 2 spare blocks
        std::vector<uint64_t> roff(N + 1, 0);
        for (uint32_t i = 0; i < N; ++i) roff[i + 1] = roff[i] + ((off[i + 1] - off[i] + 31) / 32 + 2) * 32;
        std::vector<uint32_t> rowb(roff[N] + 1, 0);
        for (uint32_t i = 0; i < N; ++i)
            for (uint64_t t = off[i]; t < off[i + 1]; ++t) rowb[roff[i] + (t - off[i])] = ids[t] * p->ndw * 4;
        size_t need = Carve::bytes_for(total + 64, 2) + Carve::bytes_for(N + 1, 8) +
                      Carve::bytes_for((uint64_t)N * p->n_sym * p->ndw, 4) + Carve::bytes_for(rowb.size(), 4) +
                      Carve::bytes_for(N + 1, 8);
        int rc = p->mem.ensure(need);
        if (rc != NMZ_OK) return cleanup(rc);
        Carve cv(p->mem.ptr);
        p->d_qsym = cv.take<uint16_t>(total + 64);
        p->d_qoff = cv.take<uint64_t>(N + 1);
        p->d_peq = cv.take<uint32_t>((uint64_t)N * p->n_sym * p->ndw);
        p->d_rowb = cv.take<uint32_t>(rowb.size());
        p->d_rowb_off = cv.take<uint64_t>(N + 1);
        if (hipMemcpyAsync(p->d_rowb, rowb.data(), rowb.size() * 4, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_rowb_off, roff.data(), (N + 1) * 8, hipMemcpyHostToDevice, st))
            return cleanup(fail(NMZ_EHIP, "ED plan upload failed"));
        if (hipMemsetAsync(p->d_qsym, 0, (total + 64) * 2, st) ||
            (total && hipMemcpyAsync(p->d_qsym, ids.data(), total * 2, hipMemcpyHostToDevice, st)) ||
            hipMemcpyAsync(p->d_qoff, off, (N + 1) * 8, hipMemcpyHostToDevice, st))
            return cleanup(fail(NMZ_EHIP, "ED plan upload failed"));
        rc = ed_wide_build_peq(p->d_qsym, p->d_qoff, N, p->n_sym, p->ndw, p->ww, p->d_peq, st);
        if (rc != NMZ_OK) return cleanup(rc);
        if (hipStreamSynchronize(st)) return cleanup(fail(NMZ_EHIP, "ED plan build failed"));
        p->dict = std::move(dict);
    } else if (fast && p->bv) {
        const uint32_t rq = ed_bv_row_queries();
        const uint32_t G = (N + rq - 1) / rq;
        p->G = G;
        p->rq = rq;
        p->maxlen = maxlen;
        p->n_sym = n_sym;
        p->dict = std::move(dict);
        const uint32_t ndw = p->ndw;
        const uint32_t zero_row = p->cmp ? n_sym : n_sym * ndw * 8;
        std::vector<uint32_t> len(N + 1, 0);
        std::vector<uint64_t> soff(N + 1, 0), chunk_start(G + 1, 0);
        for (uint32_t i = 0; i < N; ++i) {
            len[i] = (uint32_t)(off[i + 1] - off[i]);
            soff[i + 1] = soff[i] + ((uint64_t)(len[i] + 31) / 32 + 1) * 32;  // whole blocks + 1 spare
        }
        // candidates per workgroup: a larger pool amortises the Peq build and evens out the lanes' refill
        // tail, a smaller one keeps enough workgroups for small N (configs[2]-shaped traces, 1 MI355X:
        // N = 100k: 1024 -> 1.78 s, 4096 -> 1.64 s, 8192 -> 1.65 s; N = 8192: 1024 -> 14.5 ms, 4096 -> 19.6 ms)
        p->pool = p->cmp ? std::min(pool0, ED_BV_POOL) : pool0;
        for (uint32_t b = 0; b < G; ++b)
            chunk_start[b + 1] = chunk_start[b] + (N - rq * b + p->pool - 1) / p->pool;
        p->n_chunks = chunk_start[G];
        p->row_chunks.resize(G);
        for (uint32_t b = 0; b < G; ++b) p->row_chunks[b] = chunk_start[b + 1] - chunk_start[b];
        std::vector<uint16_t> bs(soff[N] + 64, (uint16_t)zero_row);  // + 2 spare blocks at the end
        for (uint32_t i = 0; i < N; ++i)
            for (uint32_t t = 0; t < len[i]; ++t)
                bs[soff[i] + t] = (uint16_t)(p->cmp ? ids[off[i] + t] : ids[off[i] + t] * ndw * 8);
        size_t need = Carve::bytes_for(bs.size(), 2) + Carve::bytes_for(N + 1, 8) * 2 +
                      Carve::bytes_for(G + 1, 8) + Carve::bytes_for(N + 1, 4) +
                      Carve::bytes_for(ED_CNT_WORDS, 8) + Carve::bytes_for((uint64_t)N * ED_QG_DW, 4);
        int rc = p->mem.ensure(need);
        if (rc != NMZ_OK) return cleanup(rc);
        Carve cv(p->mem.ptr);
        p->d_counters = cv.take<uint64_t>(ED_CNT_WORDS);
        p->d_prof = cv.take<uint32_t>((uint64_t)N * ED_QG_DW);
        p->d_bsym = cv.take<uint16_t>(bs.size());
        p->d_soff = cv.take<uint64_t>(N + 1);
        p->d_qoff = cv.take<uint64_t>(N + 1);
        p->d_chunk_start = cv.take<uint64_t>(G + 1);
        p->d_len = cv.take<uint32_t>(N + 1);
        if (hipMemcpyAsync(p->d_bsym, bs.data(), bs.size() * 2, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_soff, soff.data(), (N + 1) * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_qoff, off, (N + 1) * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_chunk_start, chunk_start.data(), (G + 1) * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_len, len.data(), (N + 1) * 4, hipMemcpyHostToDevice, st) ||
            hipMemsetAsync(p->d_counters, 0, ED_CNT_WORDS * 8, st))
            return cleanup(fail(NMZ_EHIP, "ED plan upload failed"));
        rc = ed_qgram_profiles(p->d_bsym, p->d_soff, p->d_len, N, p->d_prof, st);
        if (rc != NMZ_OK) return cleanup(rc);
        if (hipStreamSynchronize(st)) return cleanup(fail(NMZ_EHIP, "ED plan build failed"));
    } else if (fast && tile_band && maxlen + band < MAX_FAST_LEN) {
        const uint32_t G = (N + 63) / 64;
        p->G = G;
        std::vector<uint32_t> gmax(G + 1, 0), len(N + 1, 0);
        std::vector<uint64_t> coff(G + 1, 0);
        for (uint32_t i = 0; i < N; ++i) {
            len[i] = (uint32_t)(off[i + 1] - off[i]);
            gmax[i / 64] = std::max(gmax[i / 64], len[i]);
        }
        for (uint32_t g = 0; g < G; ++g) coff[g + 1] = coff[g] + (uint64_t)gmax[g] * 64;
        std::vector<uint16_t> cs(coff[G] + 1, CAND_PAD);
        for (uint32_t i = 0; i < N; ++i) {
            const uint64_t base = coff[i / 64] + (i % 64);
            for (uint32_t t = 0; t < len[i]; ++t) cs[base + (uint64_t)t * 64] = ids[off[i] + t];
        }
        size_t need = Carve::bytes_for(total + 1, 2) + Carve::bytes_for(cs.size(), 2) +
                      Carve::bytes_for(N + 1, 8) + Carve::bytes_for(G + 1, 8) + Carve::bytes_for(G + 1, 4) +
                      Carve::bytes_for(N + 1, 4);
        int rc = p->mem.ensure(need);
        if (rc != NMZ_OK) return cleanup(rc);
        Carve cv(p->mem.ptr);
        p->d_qsym = cv.take<uint16_t>(total + 1);
        p->d_csym = cv.take<uint16_t>(cs.size());
        p->d_qoff = cv.take<uint64_t>(N + 1);
        p->d_coff = cv.take<uint64_t>(G + 1);
        p->d_gmax = cv.take<uint32_t>(G + 1);
        p->d_len = cv.take<uint32_t>(N + 1);
        if ((total && hipMemcpyAsync(p->d_qsym, ids.data(), total * 2, hipMemcpyHostToDevice, st)) ||
            hipMemcpyAsync(p->d_csym, cs.data(), cs.size() * 2, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_qoff, off, (N + 1) * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_coff, coff.data(), (G + 1) * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_gmax, gmax.data(), (G + 1) * 4, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(p->d_len, len.data(), (N + 1) * 4, hipMemcpyHostToDevice, st) ||
            hipStreamSynchronize(st))
            return cleanup(fail(NMZ_EHIP, "ED plan upload failed"));
        p->dict = std::move(dict);
        p->tile = true;
    } else {
        p->fast = false;
        p->bv = false;
        p->cmp = false;
        size_t need = Carve::bytes_for(N + 1, 8) + Carve::bytes_for(total + 1, 8);
        int rc = p->mem.ensure(need);
        if (rc != NMZ_OK) return cleanup(rc);
        Carve cv(p->mem.ptr);
        p->d_off64 = cv.take<uint64_t>(N + 1);
        p->d_sym64 = cv.take<uint64_t>(total + 1);
        if (hipMemcpyAsync(p->d_off64, off, (N + 1) * 8, hipMemcpyHostToDevice, st) ||
            (total && hipMemcpyAsync(p->d_sym64, sym, total * 8, hipMemcpyHostToDevice, st)) ||
            hipStreamSynchronize(st))
            return cleanup(fail(NMZ_EHIP, "ED plan upload failed"));
    }
    *out = p;
    return NMZ_OK;
}

// Entries per DP work item. One workgroup runs one item with its pair's Peq tables; the last items of a launch
// leave CUs idle until they end, so their length is the launch's tail (~1 item per CU slot): a shard of the
// 8-GPU search has 1/8 of the items, so the tail weighs 8x more there.
uint32_t ed_bv_item() {
    if (const char *e = ab_env("NMZ_ED_ITEM")) {
        const uint32_t v = (uint32_t)atoi(e);
        if (v >= 64 && v <= ED_BV_ITEM && (v & (v - 1)) == 0) return v;
    }
    return ED_BV_ITEM;
}

// The item size of a search with n_ent DP entries: about ED_DP_ITEMS_TARGET items (8 per workgroup slot of the
// chip), a power of two in [128, ED_BV_ITEM]. Large items keep every lane busy (a lane refills from its item's
// entries as its pairs end); small ones shorten the last round of a launch, which dominates a shard's search when
// its entries are few (configs[2], 8 shards, item 4096 -> 256: clustered shard DP 9.75 -> 9.45 ms, survey 0.41-0.62
// -> 0.35-0.41 ms, profiles/r05/ed_item_ab). An NMZ_ED_ITEM setting (A/B) wins.
constexpr uint64_t ED_DP_ITEMS_TARGET = 8ull * 256 * 5;
uint32_t ed_bv_pick_item(uint64_t n_ent) {
    if (ab_env("NMZ_ED_ITEM")) return ed_bv_item();
    uint32_t it = 128;
    while (it < ED_BV_ITEM && (uint64_t)it * 2 * ED_DP_ITEMS_TARGET <= n_ent) it *= 2;
    return it;
}

// The two-phase bit-parallel search of one shard (nmz_internal.h EdQgArgs): filter count pass, scans (entry and
// work-item offsets; the two totals come back to the host to size the entry lists and the DP grid), write pass,
// DP over the work items. Returns 1 when the entry lists would exceed ED_TP_MAX_ENTRIES (caller falls back to
// the single-kernel search).
constexpr uint64_t ED_TP_MAX_ENTRIES = 1ULL << 30;  // 4 GiB of entries
constexpr uint64_t ED_TP_MAX_REC_BYTES = 1ULL << 30;

// the entry-list limit (NMZ_ED_TP_MAX_ENTRIES lowers it, so tests can force the single-kernel fallback)
static uint64_t ed_tp_max_entries() {
    if (const char *e = ab_env("NMZ_ED_TP_MAX_ENTRIES")) {
        const unsigned long long v = strtoull(e, nullptr, 10);
        if (v < ED_TP_MAX_ENTRIES) return v;
    }
    return ED_TP_MAX_ENTRIES;
}

// The two-phase search's offsets after a count pass (ed_bv_two_phase), in two launches: k_tp_reduce sums each
// block's chunk of query pairs (DP entries, work items of `item` entries), k_tp_scan turns the sums into the pairs'
// entry offsets (poff) and work-item offsets (ioff). The last block writes the 64-bit entry total (the u32 offsets
// wrap beyond 2^32 entries, so they are trusted only while the total is within the batching limit), compares the
// totals with a shard's cached sizes (flag), and moves the survivor-record counter to rec_out, leaving it at zero
// for the next count pass. (These were hipcub scans of the two arrays, an item kernel, a one-block sum, a verify
// kernel, a cursor copy and two clears: 11 launches and ~55 us per search, a fixed cost each shard of the 8-GPU
// search paid once more.)
constexpr uint32_t TP_PER_THREAD = 8, TP_TILE = 256 * TP_PER_THREAD, TP_MAX_BLOCKS = 256;
struct TpScanArgs {
    const uint32_t *cnt;    // [n] DP entries per query pair
    uint32_t n, lg_item;    // pairs; log2 entries per work item
    uint32_t chunk, nb;     // pairs per block (a multiple of TP_TILE), blocks (<= TP_MAX_BLOCKS)
    uint64_t *agg;          // [2 TP_MAX_BLOCKS]: block b's entries, items
    uint32_t *poff, *ioff;  // [n + 1]
    uint64_t *tot64;
    uint32_t *n_rec, *rec_out;  // the records' stripe counters (or nullptr) and where their total goes (UINT32_MAX
                                // when a stripe overflowed rec_share: the write pass then recomputes)
    uint32_t *rec_cnt;          // [ED_REC_STRIPES] the stripes' counts, for the scatter
    uint32_t rec_share;
    uint32_t *flag;         // or nullptr: no cached sizes to compare
    uint64_t e_tot;
    uint32_t e_items, e_rec;
    uint32_t *h_flag;       // with flag: pinned host words {seq, flag} the check publishes (ed_tp_flag_check)
    uint32_t seq;
};

__device__ __forceinline__ uint32_t tp_items(uint32_t c, uint32_t lg) { return (c + (1u << lg) - 1) >> lg; }

// block-wide sums of two u64 (256 threads); every thread gets them
__device__ __forceinline__ void tp_block_sum(uint64_t &a, uint64_t &b, uint64_t (*sh)[4]) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
        a += __shfl_xor((unsigned long long)a, off, 64);
        b += __shfl_xor((unsigned long long)b, off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        sh[0][threadIdx.x >> 6] = a;
        sh[1][threadIdx.x >> 6] = b;
    }
    __syncthreads();
    a = sh[0][0] + sh[0][1] + sh[0][2] + sh[0][3];
    b = sh[1][0] + sh[1][1] + sh[1][2] + sh[1][3];
    __syncthreads();
}

__global__ __launch_bounds__(256) void k_tp_reduce(TpScanArgs A) {
    __shared__ uint64_t sh[2][4];
    const uint32_t lo = blockIdx.x * A.chunk, hi = min(A.n, lo + A.chunk);
    uint64_t e = 0, it = 0;
    for (uint32_t i = lo + threadIdx.x; i < hi; i += 256) {
        const uint32_t c = A.cnt[i];
        e += c;
        it += tp_items(c, A.lg_item);
    }
    tp_block_sum(e, it, sh);
    if (threadIdx.x == 0) {
        A.agg[2 * blockIdx.x] = e;
        A.agg[2 * blockIdx.x + 1] = it;
    }
}

__global__ __launch_bounds__(256) void k_tp_scan(TpScanArgs A) {
    __shared__ uint64_t sh[2][4];
    const uint32_t t = threadIdx.x, lane = t & 63, wv = t >> 6;
    uint64_t ce = 0, ci = 0;  // the entries and items before this block (nb <= 256: one sum per thread)
    if (t < blockIdx.x) {
        ce = A.agg[2 * t];
        ci = A.agg[2 * t + 1];
    }
    tp_block_sum(ce, ci, sh);
    const uint32_t hi = min(A.n, (blockIdx.x + 1) * A.chunk);
    for (uint32_t base = blockIdx.x * A.chunk; base < hi; base += TP_TILE) {
        const uint32_t i0 = base + TP_PER_THREAD * t;
        uint32_t c[TP_PER_THREAD];
        if (i0 + TP_PER_THREAD <= hi) {
            const uint4 x = *(const uint4 *)(A.cnt + i0), y = *(const uint4 *)(A.cnt + i0 + 4);
            c[0] = x.x, c[1] = x.y, c[2] = x.z, c[3] = x.w, c[4] = y.x, c[5] = y.y, c[6] = y.z, c[7] = y.w;
        } else {
#pragma unroll
            for (uint32_t k = 0; k < TP_PER_THREAD; ++k) c[k] = i0 + k < hi ? A.cnt[i0 + k] : 0u;
        }
        uint64_t se = 0, si = 0;
#pragma unroll
        for (uint32_t k = 0; k < TP_PER_THREAD; ++k) {
            se += c[k];
            si += tp_items(c[k], A.lg_item);
        }
        // the thread's exclusive prefix inside the tile: wave scan, then the earlier waves' totals
        uint64_t xe = se, xi = si;
#pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
            const uint64_t ue = __shfl_up((unsigned long long)xe, d, 64), ui = __shfl_up((unsigned long long)xi, d, 64);
            if (lane >= (uint32_t)d) {
                xe += ue;
                xi += ui;
            }
        }
        if (lane == 63) {
            sh[0][wv] = xe;
            sh[1][wv] = xi;
        }
        __syncthreads();
        uint64_t pe = ce + xe - se, pi = ci + xi - si, te = 0, ti = 0;
        for (uint32_t w = 0; w < 4; ++w) {
            if (w < wv) {
                pe += sh[0][w];
                pi += sh[1][w];
            }
            te += sh[0][w];
            ti += sh[1][w];
        }
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < TP_PER_THREAD; ++k) {
            if (i0 + k < hi) {
                A.poff[i0 + k] = (uint32_t)pe;
                A.ioff[i0 + k] = (uint32_t)pi;
            }
            pe += c[k];
            pi += tp_items(c[k], A.lg_item);
        }
        ce += te;
        ci += ti;
    }
    if (blockIdx.x + 1 == A.nb && t < 64) {  // the last block's first wave: totals, record counts, the check
        uint32_t r = 0;
        bool over = false;
        if (A.n_rec) {  // (ED_REC_STRIPES == 64: a lane per stripe)
            const uint32_t c = A.n_rec[t * ED_REC_LINE];
            A.rec_cnt[t] = c;
            A.n_rec[t * ED_REC_LINE] = 0;
            over = __ballot(c > A.rec_share) != 0;
            r = c;
            for (int o = 32; o >= 1; o >>= 1) r += __shfl_xor(r, o, 64);
            if (over) r = 0xFFFFFFFFu;
        }
        if (t == 0) {
            A.poff[A.n] = (uint32_t)ce;
            A.ioff[A.n] = (uint32_t)ci;
            *A.tot64 = ce;
            if (A.n_rec) *A.rec_out = r;
            if (A.flag) {
                if (ce != A.e_tot || (uint32_t)ci != A.e_items || r != A.e_rec) atomicOr(A.flag, 1u);
                // the device flag as it now stands (sticky until reported) to the host, then the search's sequence
                // number: the host reads the flag once it sees the number (no copy, no event on the queue)
                if (A.h_flag) {
                    const uint32_t fv = __hip_atomic_load(A.flag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                    __hip_atomic_store(A.h_flag + 1, fv, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
                    __hip_atomic_store(A.h_flag, A.seq, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
                }
            }
        }
    }
}

static int tp_offsets(TpScanArgs &A, uint32_t item, hipStream_t st) {
    A.lg_item = 0;
    while ((1u << A.lg_item) < item) ++A.lg_item;
    NMZ_CHECK((1u << A.lg_item) == item, "internal: the work-item size is not a power of two");
    const uint32_t tiles = (A.n + TP_TILE - 1) / TP_TILE;
    A.nb = std::min(tiles, TP_MAX_BLOCKS);
    A.chunk = (tiles + A.nb - 1) / A.nb * TP_TILE;
    A.nb = (A.n + A.chunk - 1) / A.chunk;
    hipLaunchKernelGGL(k_tp_reduce, dim3(A.nb), dim3(256), 0, st, A);
    hipLaunchKernelGGL(k_tp_scan, dim3(A.nb), dim3(256), 0, st, A);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// The mismatch flag of searches enqueued with a shard's cached sizes (see ed_bv_two_phase). Such a search's offsets
// scan compares its totals with the cache, sets the device flag on a difference and writes {its sequence number, the
// flag as it now stands} to pinned host words (no copy or event on the queue: each was ~5-10 us per search). arm:
// mark that a search was enqueued. check: read the host words -- without waiting (the shard's next search: a number
// not yet landed is read by a later call, the device flag stays set until reported) -- or the device flag after
// synchronising `st` (wait: the synchronous entry points); when set, clear it, drop every cached size (the next
// search recounts) and fail.
int ed_tp_flag_host(nmz_ed_plan *p) {
    if (!p->h_tp_flag) {
        NMZ_HIP(hipHostMalloc((void **)&p->h_tp_flag, 8, hipHostMallocCoherent));  // device stores reach it directly
        p->h_tp_flag[0] = p->h_tp_flag[1] = 0;
        p->tp_seq = 0;
    }
    return NMZ_OK;
}

int ed_tp_flag_arm(nmz_ed_plan *p, hipStream_t) {
    if (!p->d_tp_mismatch) return NMZ_OK;
    p->tp_flag_armed = true;  // the search's scan publishes {tp_seq, flag} to h_tp_flag
    return NMZ_OK;
}

// the scan of search number `seq` has published its flag
static bool ed_tp_flag_landed(const nmz_ed_plan *p, uint32_t seq) {
    return __atomic_load_n(&p->h_tp_flag[0], __ATOMIC_ACQUIRE) == seq;
}

int ed_tp_flag_check(nmz_ed_plan *p, bool wait, hipStream_t st) {
    if (!p->d_tp_mismatch) return NMZ_OK;
    uint32_t f = 0;
    if (wait) {
        NMZ_HIP(hipMemcpyAsync(&f, p->d_tp_mismatch, 4, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
    } else {
        if (!p->tp_flag_armed || !p->h_tp_flag) return NMZ_OK;
        if (!ed_tp_flag_landed(p, p->tp_seq)) return NMZ_OK;  // not yet: a later call reads it (the flag stays set)
        f = __atomic_load_n(&p->h_tp_flag[1], __ATOMIC_ACQUIRE);
    }
    p->tp_flag_armed = false;
    if (!f) return NMZ_OK;
    NMZ_HIP(hipMemsetAsync(p->d_tp_mismatch, 0, 4, st));
    if (p->h_tp_flag) p->h_tp_flag[1] = 0;
    p->tp_sizes.clear();
    p->tp_dirty = true;  // the skipped write pass left the count pass's counts in place
    return fail(NMZ_EHIP, "internal: a two-phase search's totals differed from the shard's cached sizes; that search "
                          "wrote no entries and ran no DP (its k-NN lists are incomplete), and the cached sizes are "
                          "dropped");
}

// before the pinned flag words are freed: the last armed search's scan has written them (bounded wait, then a device
// synchronisation)
void ed_tp_flag_release(nmz_ed_plan *p) {
    if (!p->h_tp_flag) return;
    if (const uint32_t seq = p->tp_seq_sent) {
        for (int i = 0; i < 200000 && !ed_tp_flag_landed(p, seq); ++i)
            std::this_thread::sleep_for(std::chrono::microseconds(50));
        if (!ed_tp_flag_landed(p, seq)) (void)hipDeviceSynchronize();
    }
    (void)hipHostFree(p->h_tp_flag);
    p->h_tp_flag = nullptr;
}

// The shard's tiles in query-block order; the count pass sizes the entry lists. Entry lists beyond
// ed_tp_max_entries() are split: the shard's query blocks run in batches (whole blocks, at least one per batch) whose
// entries fit, each batch a count pass, scans, the write pass and the DP. Every shard of a search therefore covers
// exactly its own query blocks, whatever its entry total (a single-kernel fallback per shard deals pairs by a
// different rule, and shards that chose differently would drop or double pairs). Returns 1 only when the plan
// cannot take the two-phase search at all (N >= 2^30: entries carry j in 30 bits), the same on every shard.
static int ed_bv_two_phase(nmz_ed_plan *p, hipStream_t st, EdBvArgs &A, uint64_t *d_knn) {
    const uint32_t N = p->n, n_pairs = (N + 1) / 2, QB = (N + 63) / 64, NCB = (N + 255) / 256;
    const uint32_t shard = A.shard, n_shards = A.n_shards;
    if (N >= (1u << 30)) return 1;
    // this shard's tiles (qb << 32 | cb), built and uploaded once per (shard, n_shards): every tile of
    // query block qb belongs to shard ed_block_shard(qb). Whole query blocks, so a query pair's DP entries stay in
    // one shard's work items: dealt by tile, a pair's near-duplicate candidates (a few 256-wide tiles) spread over
    // several shards, every shard built the pair's Peq tables for a fraction of its entries, and the 8 shards
    // summed to 1.15x the unsharded search. The DP work is data-dependent and clustered (the clustered workload's
    // families put it next to the diagonal, with a period of 16 query blocks); a hash breaks that periodicity,
    // where a round-robin deal aligned with it (8 shards: max/mean shard time 1.27)
    const uint64_t key = ((uint64_t)shard << 32) | n_shards;
    DevBuf &tl = p->tile_list[key];
    // Tiles in 2-D superblocks of ED_SQ query blocks x ED_SC candidate blocks (2,048 queries x 4,096 candidates: 768
    // KiB of profiles) and the filter kernels hand each XCD a contiguous range of the list, so an XCD's L2 holds a
    // superblock's profiles while its tiles run (query-block order fetched every candidate profile once per query
    // block: 7.1 GB per launch). Batches are whole groups of ED_SQ of the shard's query blocks.
    constexpr uint32_t ED_SQ = 32, ED_SC = 16;
    std::vector<uint32_t> qbs, grp;  // the shard's query blocks; per group: first index into qbs, first tile
    auto shard_tiles = [&](std::vector<uint64_t> *tiles) {
        uint64_t t = 0;
        qbs.clear();
        grp.clear();
        for (uint32_t qb = 0; qb < QB; ++qb)
            if (ed_block_shard(qb, n_shards) == shard) qbs.push_back(qb);
        for (size_t g0 = 0; g0 < qbs.size(); g0 += ED_SQ) {
            const size_t g1 = std::min(qbs.size(), g0 + ED_SQ);
            grp.push_back((uint32_t)g0);
            grp.push_back((uint32_t)t);
            for (uint32_t cb0 = qbs[g0] / 4; cb0 < NCB; cb0 += ED_SC)
                for (size_t i = g0; i < g1; ++i)
                    for (uint32_t cb = std::max(cb0, qbs[i] / 4); cb < std::min(NCB, cb0 + ED_SC); ++cb, ++t)
                        if (tiles) tiles->push_back(((uint64_t)qbs[i] << 32) | cb);
        }
        return t;
    };
    if (!p->tile_count.count(key)) {
        std::vector<uint64_t> tiles;
        shard_tiles(&tiles);
        NMZ_TRY(tl.ensure(Carve::bytes_for(tiles.size() + 1, 8)));
        if (!tiles.empty()) NMZ_HIP(hipMemcpy(tl.ptr, tiles.data(), tiles.size() * 8, hipMemcpyHostToDevice));
        p->tile_count[key] = tiles.size();
    }
    // scratch: {mismatch flag, record count out}, the entry total, the offset kernels' block sums, the records'
    // per-stripe counts, the per-pair counts (zero between searches: the write pass takes back what the count pass
    // added) and offsets
    const size_t tp_bytes = Carve::bytes_for(4, 4) + Carve::bytes_for(1, 8) + Carve::bytes_for(2 * TP_MAX_BLOCKS, 8) +
                            Carve::bytes_for(ED_REC_STRIPES, 4) + 3 * Carve::bytes_for(n_pairs + 1, 4);
    // an earlier search of this plan whose sizes contradicted the cache is reported here (without waiting for it)
    NMZ_TRY(ed_tp_flag_check(p, false, st));
    NMZ_TRY(p->tp_mem.ensure(tp_bytes));
    Carve cv(p->tp_mem.ptr);
    uint32_t *f = cv.take<uint32_t>(4);
    uint64_t *d_tot64 = cv.take<uint64_t>(1), *d_agg = cv.take<uint64_t>(2 * TP_MAX_BLOCKS);
    uint32_t *d_rec_cnt = cv.take<uint32_t>(ED_REC_STRIPES);
    uint32_t *d_cnt = cv.take<uint32_t>(n_pairs + 1), *d_poff = cv.take<uint32_t>(n_pairs + 1);
    uint32_t *d_ioff = cv.take<uint32_t>(n_pairs + 1);
    if (p->tp_mem.gen != p->tp_mem_gen || f != p->d_tp_mismatch) {  // a new scratch buffer: flag and counts clear
        NMZ_HIP(hipMemsetAsync(p->tp_mem.ptr, 0, tp_bytes, st));
        p->d_tp_mismatch = f;
        p->tp_mem_gen = p->tp_mem.gen;
    } else if (p->tp_dirty) {  // an earlier search stopped between its count and write passes
        NMZ_HIP(hipMemsetAsync(d_cnt, 0, (n_pairs + 1) * 4, st));
    }
    const uint64_t n_tiles_all = p->tile_count[key];
    EdQgArgs Q;
    Q.prof = A.prof;
    Q.len = A.len;
    Q.knn = A.knn;
    Q.counters = A.counters;
    Q.cnt = d_cnt;
    Q.poff = d_poff;
    Q.ent = nullptr;
    Q.ent_cap = 0;
    Q.abort = f;  // the mismatch flag: the write pass and the DP skip when it is set
    // the count pass's survivor records (32 B per (wave, query pair) with survivors) let the write pass scatter
    // without recomputing the filter; room for 16 per tile, in ED_REC_STRIPES equal regions (a stripe that overflows
    // its region: the write pass recomputes)
    const uint64_t rec_cap = std::min<uint64_t>(n_tiles_all * 16, ED_TP_MAX_REC_BYTES / 32);
    // (at least 256 per stripe: a small search's few workgroups each land in one stripe, up to 128 records each)
    const uint64_t rec_share = std::max<uint64_t>((rec_cap + ED_REC_STRIPES - 1) / ED_REC_STRIPES, 256);
    constexpr size_t REC_CTR_BYTES = (size_t)ED_REC_STRIPES * ED_REC_LINE * 4;  // the stripe counters, then records
    Q.recs = nullptr;
    Q.rec_cap = 0;
    Q.rec_cnt = d_rec_cnt;
    // (NMZ_ED_QG_RECOMPUTE=1 skips the records: the recompute path, for tests)
    const char *rc_env = ab_env("NMZ_ED_QG_RECOMPUTE");
    // (the kernels count records with a u32 atomic, up to 128 per tile: a launch that could pass 2^32 of them would
    // wrap the counter, so such searches recompute instead)
    if (!(rc_env && atoi(rc_env) == 1) && n_tiles_all * 128 < (1ULL << 32) &&
        p->tp_rec.ensure(Carve::bytes_for(REC_CTR_BYTES + rec_share * ED_REC_STRIPES * 32, 1)) == NMZ_OK) {
        Q.recs = p->tp_rec.as<uint4>() + REC_CTR_BYTES / 16;
        Q.rec_cap = (uint32_t)rec_share;
    }
    Q.n_rec = Q.recs ? p->tp_rec.as<uint32_t>() : nullptr;  // the stripe counters, at the buffer's start
    // (k_tp_scan leaves them at zero; a new allocation -- tp_rec's generation changed, whatever its address -- or
    // an interrupted search clears them here)
    if (Q.n_rec && (p->tp_rec.gen != p->tp_rec_gen || p->tp_dirty)) {
        NMZ_HIP(hipMemsetAsync(Q.n_rec, 0, REC_CTR_BYTES, st));
        p->tp_rec_gen = p->tp_rec.gen;
    }
    // records in the regions (UINT32_MAX when a stripe overflowed its region)
    const uint64_t rec_total_cap = rec_share * ED_REC_STRIPES;
    Q.N = N;
    Q.k = A.k;
    Q.QB = QB;
    Q.NCB = NCB;
    Q.shard = shard;
    Q.n_shards = n_shards;
    Q.w = p->band;
    // entries per DP work item: from the search's entry total (ed_bv_pick_item) unless NMZ_ED_ITEM fixes it
    uint32_t item = ed_bv_item();
    const uint64_t limit = std::min<uint64_t>(ed_tp_max_entries(), 0xFFFFFFFFull);
    // count pass + scans over a tile list: entry and item totals
    uint32_t n_rec = 0;
    // readback = false (sizes known from an earlier search of this shard): everything stays on the device
    // the offset kernels' arguments (tp_offsets); verify = a shard's cached sizes to compare with
    auto offsets = [&](bool with_rec, const nmz_ed_plan::TpSizes *verify) -> int {
        TpScanArgs S{};
        S.cnt = d_cnt;
        S.n = n_pairs;
        S.agg = d_agg;
        S.poff = d_poff;
        S.ioff = d_ioff;
        S.tot64 = d_tot64;
        S.n_rec = with_rec ? Q.n_rec : nullptr;
        S.rec_out = f + 1;
        S.rec_cnt = d_rec_cnt;
        S.rec_share = Q.rec_cap;
        S.flag = verify ? p->d_tp_mismatch : nullptr;
        S.h_flag = verify ? p->h_tp_flag : nullptr;
        S.seq = p->tp_seq;
        if (verify) {
            // (NMZ_ED_TP_FAKE_MISMATCH=1, a test knob: compare against a wrong total, so the flag path runs)
            const char *fake = ab_env("NMZ_ED_TP_FAKE_MISMATCH");
            S.e_tot = verify->tot64 + ((fake && atoi(fake) == 1) ? 1 : 0);
            S.e_items = verify->items;
            S.e_rec = verify->n_rec;
        }
        const int rc = tp_offsets(S, item, st);
        if (rc == NMZ_OK && S.h_flag) p->tp_seq_sent = S.seq;
        return rc;
    };
    auto count = [&](const uint64_t *tiles, uint64_t n_tiles, uint64_t &tot64, uint32_t &tot_items,
                     const nmz_ed_plan::TpSizes *verify = nullptr) -> int {
        Q.tiles = tiles;
        Q.n_tiles = n_tiles;
        p->tp_dirty = true;  // until the write pass has taken the counts back
        {
            KernelTimer kt(p->ctx, st, "ed_qg_filter");
            NMZ_TRY(ed_qg_filter_launch(Q, true, st));
        }
        // the entry total in 64 bits: the u32 offsets wrap beyond 2^32 entries (about N^2 / 4 for a store of
        // near-duplicates), so they are trusted only once this total is within the limit
        NMZ_TRY(offsets(true, verify));
        if (verify) return NMZ_OK;
        NMZ_HIP(hipMemcpyAsync(&tot64, d_tot64, 8, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipMemcpyAsync(&tot_items, d_ioff + n_pairs, 4, hipMemcpyDeviceToHost, st));
        if (Q.recs) NMZ_HIP(hipMemcpyAsync(&n_rec, f + 1, 4, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        return NMZ_OK;
    };
    // write pass + DP of the tiles the last count pass covered
    auto write_dp = [&](uint64_t n_ent, uint32_t n_items) -> int {
        // the u32 scans (entry and item offsets) hold only below 2^32 entries: a batch must never reach it
        NMZ_CHECK(n_ent < (1ULL << 32), "internal: a two-phase batch reaches 2^32 entries");
        NMZ_TRY(p->tp_ent.ensure(Carve::bytes_for(n_ent + 1, 4)));
        Q.ent = p->tp_ent.as<uint32_t>();
        Q.ent_cap = n_ent;  // entry writes past the sizes the lists were made for are dropped
        {
            KernelTimer kt(p->ctx, st, "ed_qg_filter");
            if (Q.recs && n_rec <= rec_total_cap) NMZ_TRY(ed_qg_scatter_launch(Q, n_rec, st));
            else NMZ_TRY(ed_qg_filter_launch(Q, false, st));
        }
        p->tp_dirty = false;
        KernelTimer kt(p->ctx, st, "ed_bv_dp");
        return ed_bv_dp_launch(A, d_ioff, d_poff, Q.ent, n_pairs, n_items, item, p->bw, p->cmp, st, f);
    };
    uint64_t tot64 = 0;
    uint32_t tot_items = 0;
    // the DP items of the last count pass again under another item size (the first search of a shard, once its
    // entry total is known)
    auto reitem = [&](uint32_t it) -> int {
        item = it;
        NMZ_TRY(offsets(false, nullptr));
        NMZ_HIP(hipMemcpyAsync(&tot_items, d_ioff + n_pairs, 4, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        return NMZ_OK;
    };
    // The sizes the host needs before the write pass and the DP (entry total, work items, survivor records) are
    // fixed by the plan and the shard: the first search of a shard reads them back (one synchronisation), later
    // searches enqueue every kernel with those sizes and no host round trip; a one-thread kernel compares them with
    // this search's own totals and flags a difference. None can occur (the plan is immutable and the filter
    // deterministic), but if one did, the flagged search's write pass and DP skip (no write past lists sized for the
    // cached totals, no DP over offsets that disagree with them) and the shard's next search, or the next
    // synchronous call, reports it and drops the cache (ed_tp_flag_check)
    auto cached = p->tp_sizes.find(key);
    if (cached != p->tp_sizes.end() && Q.recs && cached->second.tot64 <= limit) {
        const nmz_ed_plan::TpSizes &z = cached->second;
        item = z.item;
        NMZ_TRY(ed_tp_flag_host(p));
        ++p->tp_seq;  // this search's number: its scan publishes it with the flag
        NMZ_TRY(count(tl.as<uint64_t>(), n_tiles_all, tot64, tot_items, &z));
        n_rec = z.n_rec;
        NMZ_TRY(write_dp(z.tot64, z.items));
        return ed_tp_flag_arm(p, st);
    }
    NMZ_TRY(count(tl.as<uint64_t>(), n_tiles_all, tot64, tot_items));
    if (tot64 <= limit) {
        const uint32_t it = ed_bv_pick_item(tot64);
        if (it != item) NMZ_TRY(reitem(it));
        if (Q.recs && n_rec <= rec_total_cap) p->tp_sizes[key] = nmz_ed_plan::TpSizes{tot64, tot_items, n_rec, item};
        return write_dp(tot64, tot_items);
    }
    // batches of whole query blocks: per-block totals from this count pass, then the lists and counters start over
    // (the count pass lists pairs with an empty trace, and adds to the counters)
    std::vector<uint32_t> cnt(n_pairs);
    NMZ_HIP(hipMemcpy(cnt.data(), d_cnt, (size_t)n_pairs * 4, hipMemcpyDeviceToHost));
    NMZ_HIP(hipMemsetAsync(d_cnt, 0, (n_pairs + 1) * 4, st));  // (no write pass took this count pass's counts)
    shard_tiles(nullptr);
    const size_t ng = grp.size() / 2;
    hipLaunchKernelGGL(k_knn_init, dim3(ceil_div((uint64_t)N * A.k, 256)), dim3(256), 0, st, d_knn, (uint64_t)N * A.k);
    NMZ_HIP(hipMemsetAsync(p->d_counters, 0, ED_CNT_WORDS * 8, st));
    // a query block's entry total (this count pass's per-pair counts)
    auto block_entries = [&](size_t i) {
        uint64_t c = 0;
        for (uint32_t pp = 32 * qbs[i]; pp < std::min(32 * qbs[i] + 32, n_pairs); ++pp) c += cnt[pp];
        return c;
    };
    DevBuf sub;  // the tile list of a batch narrower than one group (uploaded per batch)
    struct R3 {
        DevBuf &b;
        ~R3() { b.release(); }
    } rel_sub{sub};
    for (size_t b0 = 0; b0 < ng;) {
        uint64_t acc = 0;
        size_t b1 = b0;
        while (b1 < ng) {
            const size_t i1 = b1 + 1 < ng ? grp[2 * (b1 + 1)] : qbs.size();
            uint64_t c = 0;
            for (size_t i = grp[2 * b1]; i < i1; ++i) c += block_entries(i);
            if (acc + c > limit) break;
            acc += c;
            ++b1;
        }
        if (b1 > b0) {  // whole groups: their tiles are one contiguous range of the shard's list
            const uint64_t t0 = grp[2 * b0 + 1], t1 = b1 < ng ? grp[2 * b1 + 1] : n_tiles_all;
            NMZ_TRY(count(tl.as<uint64_t>() + t0, t1 - t0, tot64, tot_items));
            NMZ_TRY(write_dp(tot64, tot_items));
            b0 = b1;
            continue;
        }
        // one group alone exceeds the limit: its query blocks in sub-batches, each with its own tile list (the
        // group's superblock order, restricted to the sub-batch's blocks); a single block cannot be split further:
        // it runs alone, and fails loudly only at 2^32 entries (64 queries x N candidates: N >= 2^26)
        const size_t i0 = grp[2 * b0], i1 = b0 + 1 < ng ? grp[2 * (b0 + 1)] : qbs.size();
        for (size_t j0 = i0; j0 < i1;) {
            uint64_t a = 0;
            size_t j1 = j0;
            while (j1 < i1 && (j1 == j0 || a + block_entries(j1) <= limit)) a += block_entries(j1++);
            // (a block alone may pass the batching limit; it must stay below the u32 scans' 2^32)
            NMZ_CHECK(a < (1ULL << 32), "one query block's candidate entries reach 2^32 (too many traces)");
            std::vector<uint64_t> tiles;
            for (uint32_t cb0 = qbs[j0] / 4; cb0 < NCB; cb0 += ED_SC)
                for (size_t i = j0; i < j1; ++i)
                    for (uint32_t cb = std::max(cb0, qbs[i] / 4); cb < std::min(NCB, cb0 + ED_SC); ++cb)
                        tiles.push_back(((uint64_t)qbs[i] << 32) | cb);
            NMZ_TRY(sub.ensure(Carve::bytes_for(tiles.size() + 1, 8)));
            NMZ_HIP(hipStreamSynchronize(st));  // the previous sub-batch's kernels have read the list
            if (!tiles.empty())
                NMZ_HIP(hipMemcpy(sub.ptr, tiles.data(), tiles.size() * 8, hipMemcpyHostToDevice));
            NMZ_TRY(count(sub.as<uint64_t>(), tiles.size(), tot64, tot_items));
            NMZ_TRY(write_dp(tot64, tot_items));
            j0 = j1;
        }
        b0 = b0 + 1;
    }
    return NMZ_OK;
}

static int ed_knn_run(nmz_ed_plan *p, hipStream_t st, uint32_t k, uint64_t *d_knn, uint32_t shard = 0,
                      uint32_t n_shards = 1) {
    const uint32_t N = p->n;
    if (N == 0 || k == 0) return NMZ_OK;
    {
        uint64_t *cnt = p->bv ? p->d_counters : nullptr;  // zeroed with the lists (was a memset per search)
        const uint64_t nl = (uint64_t)N * k, nt = std::max<uint64_t>(nl, cnt ? ED_CNT_WORDS : 0);
        hipLaunchKernelGGL(k_knn_init_cnt, dim3(ceil_div(nt, 256)), dim3(256), 0, st, d_knn, nl, cnt,
                           (uint32_t)ED_CNT_WORDS);
    }
    if (p->wide) {
        EdWideArgs A;
        A.sym = p->d_qsym;
        A.off = p->d_qoff;
        A.rowb = p->d_rowb;
        A.rowb_off = p->d_rowb_off;
        A.peq = p->d_peq;
        A.knn = d_knn;
        A.n_pairs = (uint64_t)N * (N - 1) / 2;
        const uint64_t chunks = (A.n_pairs + 31) / 32;
        A.n_waves = (shard < chunks ? (chunks - shard + n_shards - 1) / n_shards : 0) * 32;
        A.N = N;
        A.k = k;
        A.n_sym = p->n_sym;
        A.ndw = p->ndw;
        A.shard = shard;
        A.n_shards = n_shards;
        A.w = p->band;
        if (A.n_waves == 0) return NMZ_OK;
        KernelTimer kt(p->ctx, st, "ed_wide");
        return ed_wide_launch(A, p->ww, st);
    }
    if (p->bv) {
        EdBvArgs A;
        A.bsym = p->d_bsym;
        A.soff = p->d_soff;
        A.len = p->d_len;
        A.chunk_start = p->d_chunk_start;
        A.knn = d_knn;
        A.counters = p->d_counters;
        A.prof = p->qgram ? (const uint4 *)p->d_prof : nullptr;
        A.N = N;
        A.G = p->G;
        A.k = k;
        A.lds_dw = p->lds_dw;
        A.pool = p->pool;
        A.w = p->band;
        A.rmap_dw = p->rmap_dw;
        A.claim_dw = p->claim_dw;
        A.row_bytes = p->row_bytes;
        A.shard = shard;
        A.n_shards = n_shards;
        int rc = 1;
        if (A.prof && p->two_phase) {  // filter tiles + DP work items (the search's "ed_bv" time)
            KernelTimer kt(p->ctx, st, "ed_bv");
            rc = ed_bv_two_phase(p, st, A, d_knn);
            if (rc < 0) return rc;
        }
        if (rc == 1) {  // the single-kernel search (no q-gram filter, or N >= 2^30): a plan-wide choice
            // every (row, chunk) of the plan is launched; a workgroup whose query block this shard does not own
            // (ed_block_shard, the two-phase search's rule) exits at once, so a shard owns the same pairs whichever
            // form of the search its plan took
            A.n_chunks = p->n_chunks;
            if (A.n_chunks > 0) {
                A.rq = p->rq;
                uint64_t blocks = A.n_chunks * (p->rq / 2);
                blocks = (blocks + 7) / 8 * 8;
                NMZ_CHECK(blocks < (1ULL << 31), "too many traces for one launch");
                NMZ_HIP(hipMemsetAsync(p->d_counters, 0, ED_CNT_WORDS * 8, st));
                KernelTimer kt(p->ctx, st, "ed_bv");
                NMZ_TRY(ed_bv_launch(A, p->bw, p->cmp, blocks, st));
            }
        }
        // k_ed_bv lists in-band results only; a shard's partial lists are completed after the merge
        // (nmz_ed_knn_fill_dev)
        if (n_shards == 1) {
            hipLaunchKernelGGL(k_knn_fill, dim3(ceil_div(N, 256)), dim3(256), 0, st, d_knn, N, k, N, p->band + 1, 1);
            NMZ_HIP(hipGetLastError());
        }
        return NMZ_OK;
    }
    if (p->fast) {
        EdArgs A;
        A.qsym = p->d_qsym;
        A.qoff = p->d_qoff;
        A.csym = p->d_csym;
        A.coff = p->d_coff;
        A.gmax = p->d_gmax;
        A.len = p->d_len;
        A.N = N;
        A.G = p->G;
        A.k = k;
        A.knn = d_knn;
        const uint64_t groups = tri_prefix(p->G, p->G) / 32;
        A.shard = shard;
        A.n_shards = n_shards;
        A.n_waves = (shard < groups ? (groups - shard + n_shards - 1) / n_shards : 0) * 32;
        if (A.n_waves == 0) return NMZ_OK;
        uint64_t blocks = (A.n_waves + 3) / 4;
        blocks = (blocks + 7) / 8 * 8;  // multiple of 8 for the XCD remap
        NMZ_CHECK(blocks < (1ULL << 31), "too many traces for one launch");
        KernelTimer kt(p->ctx, st, "ed_tile");
        switch (p->band) {
            case 8: hipLaunchKernelGGL(k_ed_tile<8>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
            case 16: hipLaunchKernelGGL(k_ed_tile<16>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
            case 32: hipLaunchKernelGGL(k_ed_tile<32>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
            default: return fail(NMZ_EINVAL, "internal: band has no fast kernel");
        }
        NMZ_HIP(hipGetLastError());
        return NMZ_OK;
    }
    // generic fallback: upper-triangle pair list in chunks
    const uint64_t total_pairs = (uint64_t)N * (N - 1) / 2;
    const uint64_t chunk = std::min<uint64_t>(total_pairs, 1ULL << 22);
    const unsigned gthreads = 256 * 1024;
    DevBuf &scr = p->ctx->buf[3];
    NMZ_TRY(scr.ensure(Carve::bytes_for(chunk * 2 + 1, 4) + Carve::bytes_for(chunk + 1, 4) +
                       Carve::bytes_for((uint64_t)(2 * p->band + 1) * gthreads, 4)));
    Carve cv(scr.ptr);
    uint32_t *d_pairs = cv.take<uint32_t>(chunk * 2 + 1);
    uint32_t *d_dist = cv.take<uint32_t>(chunk + 1);
    uint32_t *d_row = cv.take<uint32_t>((uint64_t)(2 * p->band + 1) * gthreads);
    for (uint64_t s = (uint64_t)shard * chunk; s < total_pairs; s += (uint64_t)n_shards * chunk) {
        const uint64_t c = std::min(chunk, total_pairs - s);
        hipLaunchKernelGGL(k_pairs_upper, dim3(ceil_div(c, 256)), dim3(256), 0, st, N, s, c, d_pairs);
        hipLaunchKernelGGL(k_ed_generic, dim3(gthreads / 256), dim3(256), 0, st, p->d_off64, p->d_sym64, d_pairs, c,
                           p->band, d_row, d_dist);
        hipLaunchKernelGGL(k_knn_from_pairs, dim3(ceil_div(c, 256)), dim3(256), 0, st, d_pairs, d_dist, c, d_knn, k);
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz

using namespace nmz;

extern "C" {

int nmz_ed_plan_create(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t n_traces, uint32_t band,
                       nmz_ed_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return ed_plan_build(ctx, off, sym, n_traces, band, out);
}

int nmz_ed_plan_destroy(nmz_ed_plan *plan) {
    if (!plan) return NMZ_OK;
    {
        CtxGuard g(plan->ctx);
        plan->mem.release();
        plan->tp_mem.release();
        plan->tp_ent.release();
        plan->tp_rec.release();
        for (auto &kv : plan->tile_list) kv.second.release();
        ed_tp_flag_release(plan);
    }
    delete plan;
    return NMZ_OK;
}

int nmz_ed_plan_is_fast(const nmz_ed_plan *plan) {
    if (!plan) return 0;
    return plan->wide ? 3 : (plan->bv ? 2 : (plan->fast ? 1 : 0));
}

int nmz_debug_tp_offsets(nmz_ctx *ctx, const uint32_t *d_cnt, uint32_t n, uint32_t item, uint32_t *d_poff,
                         uint32_t *d_ioff, uint64_t *d_tot, void *stream) {
    NMZ_CHECK(ctx != nullptr && d_cnt != nullptr && d_poff != nullptr && d_ioff != nullptr && d_tot != nullptr,
              "NULL argument");
    NMZ_CHECK(n > 0 && n < (1u << 30), "n out of range");
    NMZ_CHECK(item > 0 && (item & (item - 1)) == 0, "item must be a power of two");
    NMZ_CHECK(((uintptr_t)d_cnt & 15) == 0, "d_cnt must be 16-byte aligned (the scan loads uint4)");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    DevBuf agg;
    struct R {
        DevBuf &b;
        ~R() { b.release(); }
    } rel{agg};
    NMZ_TRY(agg.ensure(2 * TP_MAX_BLOCKS * 8));
    TpScanArgs S{};
    S.cnt = d_cnt;
    S.n = n;
    S.agg = agg.as<uint64_t>();
    S.poff = d_poff;
    S.ioff = d_ioff;
    S.tot64 = d_tot;
    NMZ_TRY(tp_offsets(S, item, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_ed_plan_counters(nmz_ed_plan *plan, uint64_t *out, void *stream) {
    NMZ_CHECK(plan != nullptr && out != nullptr, "NULL argument");
    for (int i = 0; i < NMZ_ED_NCOUNTERS; ++i) out[i] = 0;
    if (!plan->d_counters) return NMZ_OK;
    static_assert(ED_BV_NCOUNTERS == NMZ_ED_NCOUNTERS, "counter layout");
    CtxGuard g(plan->ctx);
    hipStream_t st = stream ? (hipStream_t)stream : plan->ctx->stream;
    std::vector<uint64_t> lines(ED_CNT_WORDS);
    NMZ_HIP(hipMemcpyAsync(lines.data(), plan->d_counters, ED_CNT_WORDS * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    for (uint32_t sidx = 0; sidx < ED_CNT_STRIPES; ++sidx)
        for (int i = 0; i < ED_BV_NCOUNTERS; ++i) out[i] += lines[sidx * ED_CNT_LINE + i];
    return ed_tp_flag_check(plan, true, st);
}

}  // extern "C"

namespace nmz {

// k_ed_query_generic over the resident store (soff/slen/sym as the kernel takes them) for n_q queries whose
// symbols (already in the store's encoding) are at d_qs + qstart[q], lengths qlen[q] (host arrays)
static int ed_query_generic_launch(nmz_ed_plan *plan, const uint64_t *soff, const uint32_t *slen, const void *sym,
                                   bool wide_sym, const void *d_qs, const std::vector<uint64_t> &qstart,
                                   const std::vector<uint32_t> &qlen, uint64_t *d_knn, uint32_t k) {
    hipStream_t st = plan->ctx->stream;
    const uint32_t N = plan->n, W = plan->band, n_q = (uint32_t)qlen.size();
    const unsigned threads =
        (unsigned)std::max<uint64_t>(256, std::min<uint64_t>(256 * 1024, (1ULL << 28) / (2ULL * W + 1)) / 256 * 256);
    DevBuf &scr = plan->ctx->buf[15];
    NMZ_TRY(scr.ensure(Carve::bytes_for(n_q + 1, 8) + Carve::bytes_for(n_q + 1, 4) +
                       Carve::bytes_for((uint64_t)(2 * W + 1) * threads, 4)));
    Carve cv(scr.ptr);
    uint64_t *d_qstart = cv.take<uint64_t>(n_q + 1);
    uint32_t *d_qlen = cv.take<uint32_t>(n_q + 1);
    uint32_t *d_row = cv.take<uint32_t>((uint64_t)(2 * W + 1) * threads);
    NMZ_HIP(hipMemcpyAsync(d_qstart, qstart.data(), n_q * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_qlen, qlen.data(), n_q * 4, hipMemcpyHostToDevice, st));
    KernelTimer kt(plan->ctx, st, "ed_query_generic");
    hipLaunchKernelGGL(k_ed_query_generic, dim3(threads / 256), dim3(256), 0, st, soff, slen, sym, wide_sym, d_qstart,
                       d_qlen, d_qs, n_q, N, W, k, d_row, d_knn);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipStreamSynchronize(st));  // pageable sources
    return NMZ_OK;
}

// nmz_ed_plan_query_knn on a bit-parallel plan: k_ed_bv_query, two queries per launch
static int ed_query_bv(nmz_ed_plan *plan, const uint64_t *q_off, const uint64_t *q_sym, uint32_t n_queries,
                       uint32_t k, uint64_t *d_knn) {
    hipStream_t st = plan->ctx->stream;
    const uint32_t N = plan->n;
    // query streams in the plan's Peq-row offsets (unknown symbols: 0xffff), each padded by one 32-block
    std::vector<uint64_t> qoff(n_queries + 1, 0);
    for (uint32_t q = 0; q < n_queries; ++q) qoff[q + 1] = qoff[q] + (q_off[q + 1] - q_off[q] + 31) / 32 * 32 + 32;
    std::vector<uint16_t> qs(qoff[n_queries] + 1, 0xffffu);
    for (uint32_t q = 0; q < n_queries; ++q)
        for (uint64_t t = q_off[q]; t < q_off[q + 1]; ++t) {
            auto it = plan->dict.find(q_sym[t]);
            if (it != plan->dict.end())
                qs[qoff[q] + (t - q_off[q])] = (uint16_t)(plan->cmp ? it->second : it->second * plan->ndw * 8);
        }
    // compact tables: each launch's rows = the two queries' distinct known symbols
    std::vector<uint32_t> qd(n_queries, 0);
    if (plan->cmp) {
        std::vector<uint32_t> stamp(plan->n_sym + 1, UINT32_MAX);
        for (uint32_t q = 0; q < n_queries; ++q)
            for (uint64_t t = qoff[q]; t < qoff[q] + (q_off[q + 1] - q_off[q]); ++t)
                if (qs[t] != 0xffffu && stamp[qs[t]] != q) {
                    stamp[qs[t]] = q;
                    ++qd[q];
                }
    }
    DevBuf &scr = plan->ctx->buf[13];
    NMZ_TRY(scr.ensure(Carve::bytes_for(qs.size(), 2)));
    uint16_t *d_qs = scr.as<uint16_t>();
    NMZ_HIP(hipMemcpyAsync(d_qs, qs.data(), qs.size() * 2, hipMemcpyHostToDevice, st));
    std::vector<uint32_t> spill;  // queries for the generic kernel
    // a pool of 256 stored traces per workgroup: one pass of lanes, ~N/256 workgroups
    const uint32_t pool = N >= 256u * 1024u ? 1024u : 256u;
    for (uint32_t q = 0; q < n_queries && N; q += 2) {
        const uint32_t nq2 = std::min(2u, n_queries - q);
        bool longq = false;  // a query longer than the Peq tables (the longest stored trace): generic kernel
        for (uint32_t i = 0; i < nq2; ++i) longq |= q_off[q + i + 1] - q_off[q + i] > plan->maxlen;
        if (longq) {
            for (uint32_t i = 0; i < nq2; ++i) spill.push_back(q + i);
            continue;
        }
        EdBvQueryArgs A;
        A.bsym = plan->d_bsym;
        A.soff = plan->d_soff;
        A.len = plan->d_len;
        A.qs = d_qs;
        A.n_queries = std::min(2u, n_queries - q);
        for (uint32_t i = 0; i < 2; ++i) {
            const uint32_t qq = std::min(q + i, n_queries - 1);
            A.qoff[i] = qoff[qq];
            A.nq[i] = (uint32_t)(q_off[qq + 1] - q_off[qq]);
        }
        A.knn = d_knn + (uint64_t)q * k;
        A.prof = plan->qgram ? (const uint4 *)plan->d_prof : nullptr;
        A.N = N;
        A.k = k;
        A.lds_dw = plan->lds_dw;
        A.pool = pool;
        A.w = plan->band;
        A.rmap_dw = plan->rmap_dw;
        A.claim_dw = plan->claim_dw;
        A.row_bytes = plan->row_bytes;
        if (plan->cmp) {
            const uint32_t R = qd[q] + (A.n_queries > 1 ? qd[q + 1] : 0);
            if (!bv_compact_layout(plan->n_sym, R, plan->ndw, 16 + (2 * ED_QG_DW + 2 * ED_QG_BUCKETS) * 4,
                                   ED_BV_LDS_MAX, A.lds_dw, A.rmap_dw, A.claim_dw)) {
                // the pair's symbols overflow the compact tables: these queries take the generic kernel over the
                // same encoded streams (below)
                for (uint32_t i = 0; i < A.n_queries; ++i) spill.push_back(q + i);
                continue;
            }
        }
        KernelTimer kt(plan->ctx, st, "ed_bv_query");
        NMZ_TRY(ed_bv_query_launch(A, plan->bw, plan->cmp, ceil_div(N, pool), st));
    }
    // stored trace j: stream at d_bsym + soff[j], d_len[j] symbols, in the same encoding as qs (an unseen query
    // symbol, 0xffff, equals no stored entry: row byte offsets are even, compact ids < 0xfffe)
    for (const uint32_t q : spill) {
        std::vector<uint64_t> qstart{qoff[q]};
        std::vector<uint32_t> qlen{(uint32_t)(q_off[q + 1] - q_off[q])};
        NMZ_TRY(ed_query_generic_launch(plan, plan->d_soff, plan->d_len, plan->d_bsym, false, d_qs, qstart, qlen,
                                        d_knn + (uint64_t)q * k, k));
    }
    NMZ_HIP(hipStreamSynchronize(st));  // the host vectors are pageable
    return NMZ_OK;
}

// nmz_ed_plan_query_knn on a wide plan: each query's match table over the store's alphabet (one more row for symbols
// the store has never seen), then k_ed_wide_query over (query, stored trace) waves; tables in batches of <= 2 GiB
static int ed_query_wide(nmz_ed_plan *plan, const uint64_t *q_off, const uint64_t *q_sym, uint32_t n_queries,
                         uint32_t k, uint64_t *d_knn) {
    hipStream_t st = plan->ctx->stream;
    const uint32_t N = plan->n, ns1 = plan->n_sym + 1, ndw = plan->ndw;
    const uint64_t tbl = (uint64_t)ns1 * ndw;  // dwords per query table
    const uint32_t batch = (uint32_t)std::max<uint64_t>(1, std::min<uint64_t>(n_queries, (2ULL << 30) / (tbl * 4)));
    uint64_t maxq = 0;
    for (uint32_t q = 0; q < n_queries; ++q)
        maxq = std::max<uint64_t>(maxq, std::min<uint64_t>(q_off[q + 1] - q_off[q], plan->maxlen));
    DevBuf &scr = plan->ctx->buf[13];
    NMZ_TRY(scr.ensure(Carve::bytes_for(batch * tbl, 4) + Carve::bytes_for(batch * maxq + 64, 2) +
                       Carve::bytes_for(batch + 1, 8) + Carve::bytes_for(batch, 4)));
    Carve cv(scr.ptr);
    uint32_t *d_tbl = cv.take<uint32_t>(batch * tbl);
    uint16_t *d_ids = cv.take<uint16_t>(batch * maxq + 64);
    uint64_t *d_qoff = cv.take<uint64_t>(batch + 1);
    uint32_t *d_qlen = cv.take<uint32_t>(batch);
    auto ids_of = [&](uint64_t b0, uint64_t n, std::vector<uint16_t> &ids, uint16_t unseen) {
        ids.resize(n);
        for (uint64_t t = 0; t < n; ++t) {
            auto it = plan->dict.find(q_sym[b0 + t]);
            ids[t] = (uint16_t)(it != plan->dict.end() ? it->second : unseen);
        }
    };
    // queries [q0, q0 + nb), each within the tables
    auto run = [&](uint32_t q0, uint32_t nb) -> int {
        const uint64_t b0 = q_off[q0], nsym = q_off[q0 + nb] - b0;
        std::vector<uint16_t> ids;
        std::vector<uint64_t> qo(nb + 1);
        std::vector<uint32_t> ql(nb);
        ids_of(b0, nsym, ids, (uint16_t)plan->n_sym);  // unseen: the spare row
        for (uint32_t q = 0; q <= nb; ++q) qo[q] = q_off[q0 + q] - b0;
        for (uint32_t q = 0; q < nb; ++q) ql[q] = (uint32_t)(qo[q + 1] - qo[q]);
        if (nsym) NMZ_HIP(hipMemcpyAsync(d_ids, ids.data(), nsym * 2, hipMemcpyHostToDevice, st));
        NMZ_HIP(hipMemcpyAsync(d_qoff, qo.data(), (nb + 1) * 8, hipMemcpyHostToDevice, st));
        NMZ_HIP(hipMemcpyAsync(d_qlen, ql.data(), nb * 4, hipMemcpyHostToDevice, st));
        NMZ_TRY(ed_wide_build_peq(d_ids, d_qoff, nb, ns1, ndw, plan->ww, d_tbl, st));
        EdWideArgs A;
        A.sym = plan->d_qsym;
        A.off = plan->d_qoff;
        A.rowb = plan->d_rowb;
        A.rowb_off = plan->d_rowb_off;
        A.peq = nullptr;
        A.knn = d_knn + (uint64_t)q0 * k;
        A.n_pairs = (uint64_t)nb * N;
        A.n_waves = A.n_pairs;
        A.N = N;
        A.k = k;
        A.n_sym = ns1;
        A.ndw = ndw;
        A.shard = 0;
        A.n_shards = 1;
        A.w = plan->band;
        KernelTimer kt(plan->ctx, st, "ed_wide_query");
        NMZ_TRY(ed_wide_query_launch(A, plan->ww, d_tbl, tbl, d_qlen, nb, st));
        NMZ_HIP(hipStreamSynchronize(st));  // the host vectors are pageable and the tables are reused
        return NMZ_OK;
    };
    uint32_t q0 = 0;
    for (uint32_t q = 0; q <= n_queries; ++q) {
        const bool end = q == n_queries, longq = !end && q_off[q + 1] - q_off[q] > plan->maxlen;
        if ((end || longq || q - q0 == batch) && q > q0) NMZ_TRY(run(q0, q - q0));
        if (longq) {  // longer than the tables: the generic kernel over the plan's dense ids (unseen: 0xffff)
            std::vector<uint16_t> ids;
            const uint64_t n = q_off[q + 1] - q_off[q];
            ids_of(q_off[q], n, ids, 0xffff);
            DevBuf one;
            struct R {
                DevBuf &b;
                ~R() { b.release(); }
            } rel{one};
            NMZ_TRY(one.ensure(Carve::bytes_for(n + 1, 2)));
            NMZ_HIP(hipMemcpyAsync(one.ptr, ids.data(), n * 2, hipMemcpyHostToDevice, st));
            NMZ_TRY(ed_query_generic_launch(plan, plan->d_qoff, nullptr, plan->d_qsym, false, one.ptr,
                                            std::vector<uint64_t>{0}, std::vector<uint32_t>{(uint32_t)n},
                                            d_knn + (uint64_t)q * k, k));
        }
        if (end || longq || q - q0 == batch) q0 = longq ? q + 1 : q;
    }
    return NMZ_OK;
}

// nmz_ed_plan_query_knn on the other plans (k_ed_tile's dense ids, or the generic plan's u64 symbols)
static int ed_query_generic(nmz_ed_plan *plan, const uint64_t *q_off, const uint64_t *q_sym, uint32_t n_queries,
                            uint32_t k, uint64_t *d_knn) {
    hipStream_t st = plan->ctx->stream;
    const bool dense = plan->tile;  // dense u16 ids (unseen query symbols: 0xffff, never a stored id)
    static_assert(MAX_FAST_SYMBOLS <= 0xffff, "0xffff must not be a dense id");
    const uint64_t total = q_off[n_queries];
    DevBuf &scr = plan->ctx->buf[13];
    NMZ_TRY(scr.ensure(Carve::bytes_for(total + 1, dense ? 2 : 8)));
    void *d_qs = scr.ptr;
    std::vector<uint16_t> ids;
    if (dense) {
        ids.resize(total);
        for (uint64_t t = 0; t < total; ++t) {
            auto it = plan->dict.find(q_sym[t]);
            ids[t] = it != plan->dict.end() ? (uint16_t)it->second : (uint16_t)0xffff;
        }
        if (total) NMZ_HIP(hipMemcpyAsync(d_qs, ids.data(), total * 2, hipMemcpyHostToDevice, st));
    } else if (total) {
        NMZ_HIP(hipMemcpyAsync(d_qs, q_sym, total * 8, hipMemcpyHostToDevice, st));
    }
    std::vector<uint64_t> qstart(n_queries);
    std::vector<uint32_t> qlen(n_queries);
    for (uint32_t q = 0; q < n_queries; ++q) {
        qstart[q] = q_off[q];
        qlen[q] = (uint32_t)(q_off[q + 1] - q_off[q]);
    }
    return ed_query_generic_launch(plan, dense ? plan->d_qoff : plan->d_off64,
                                   nullptr, dense ? (const void *)plan->d_qsym : (const void *)plan->d_sym64, !dense,
                                   d_qs, qstart, qlen, d_knn, k);
}

}  // namespace nmz

extern "C" {

int nmz_ed_plan_query_knn(nmz_ed_plan *plan, const uint64_t *q_off, const uint64_t *q_sym, uint32_t n_queries,
                          uint32_t k, uint32_t *knn_id, uint32_t *knn_dist) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    NMZ_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
    NMZ_CHECK(n_queries == 0 || (q_off && knn_id && knn_dist), "NULL argument");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    if (n_queries == 0) return NMZ_OK;
    const uint64_t total = q_off[n_queries];
    NMZ_CHECK(total == 0 || q_sym, "q_sym is NULL");
    for (uint32_t q = 0; q < n_queries; ++q) NMZ_CHECK(q_off[q] <= q_off[q + 1], "query offsets must not decrease");
    hipStream_t st = plan->ctx->stream;
    const uint32_t N = plan->n;
    const uint64_t nk = (uint64_t)n_queries * k;
    DevBuf &scr = plan->ctx->buf[11];
    NMZ_TRY(scr.ensure(Carve::bytes_for(nk, 8) + 2 * Carve::bytes_for(nk, 4)));
    Carve cv(scr.ptr);
    uint64_t *d_knn = cv.take<uint64_t>(nk);
    uint32_t *d_id = cv.take<uint32_t>(nk), *d_ds = cv.take<uint32_t>(nk);
    hipLaunchKernelGGL(k_knn_init, dim3(ceil_div(nk, 256)), dim3(256), 0, st, d_knn, nk);
    if (N) {
        if (plan->bv) NMZ_TRY(ed_query_bv(plan, q_off, q_sym, n_queries, k, d_knn));
        else if (plan->wide) NMZ_TRY(ed_query_wide(plan, q_off, q_sym, n_queries, k, d_knn));
        else NMZ_TRY(ed_query_generic(plan, q_off, q_sym, n_queries, k, d_knn));
    }
    // the query kernels list in-band results only: every other stored trace is at band + 1
    hipLaunchKernelGGL(k_knn_fill, dim3(ceil_div(n_queries, 256)), dim3(256), 0, st, d_knn, n_queries, k, N,
                       plan->band + 1, 0);
    hipLaunchKernelGGL(k_knn_final, dim3(ceil_div(nk, 256)), dim3(256), 0, st, d_knn, nk, d_id, d_ds);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipMemcpyAsync(knn_id, d_id, nk * 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipMemcpyAsync(knn_dist, d_ds, nk * 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_ed_plan_create_dev(nmz_ctx *ctx, const uint64_t *off, const uint64_t *d_sym, uint32_t n_traces,
                           uint32_t band, nmz_ed_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_traces == 0 || off, "off is NULL");
    NMZ_CHECK(n_traces == 0 || off[n_traces] == 0 || d_sym, "d_sym is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return ed_plan_build(ctx, off, nullptr, n_traces, band, out, d_sym);
}

int nmz_ed_plan_create_opts(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint64_t *d_sym,
                            uint32_t n_traces, uint32_t band, uint32_t opts, nmz_ed_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_traces == 0 || off, "off is NULL");
    NMZ_CHECK(!(sym && d_sym), "pass sym (host) or d_sym (device), not both");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return ed_plan_build(ctx, off, sym, n_traces, band, out, d_sym, opts);
}

int nmz_ed_plan_fingerprint(const nmz_ed_plan *p, uint64_t *fp) {
    NMZ_CHECK(p != nullptr && fp != nullptr, "NULL argument");
    const uint64_t kind = p->wide ? 3 : (p->bv ? 2 : (p->fast ? 1 : 0));
    fp[0] = NMZ_ED_FP_VERSION;
    fp[1] = kind | (uint64_t)p->band << 8 | (uint64_t)(p->bv ? p->bw : p->ww) << 40;
    fp[2] = p->n;
    fp[3] = p->total;
    fp[4] = (uint64_t)p->two_phase | (uint64_t)p->qgram << 1 | (uint64_t)p->cmp << 2;
    fp[5] = (uint64_t)p->rq | (uint64_t)p->pool << 32;
    fp[6] = p->off_hash;
    fp[7] = p->n_sym;
    return NMZ_OK;
}

int nmz_ed_allpairs_knn_dev(nmz_ed_plan *plan, uint32_t k, uint64_t *d_knn_keys, void *stream) {
    return nmz_ed_allpairs_knn_shard_dev(plan, k, 0, 1, d_knn_keys, stream);
}

uint32_t nmz_ed_block_shard(uint32_t qb, uint32_t n_shards) { return ed_block_shard(qb, n_shards); }

int nmz_ed_allpairs_knn_shard_dev(nmz_ed_plan *plan, uint32_t k, uint32_t shard, uint32_t n_shards,
                                  uint64_t *d_knn_keys, void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    NMZ_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
    NMZ_CHECK(n_shards >= 1 && shard < n_shards, "bad shard");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    return ed_knn_run(plan, stream ? (hipStream_t)stream : plan->ctx->stream, k, d_knn_keys, shard, n_shards);
}

// merge n_parts partial k-NN key lists ([n_parts][N][k], each sorted) into [N][k]
__global__ void k_knn_merge(const uint64_t *__restrict__ parts, uint32_t n_parts, uint32_t N, uint32_t k,
                            uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    uint32_t pos[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (uint32_t s = 0; s < k; ++s) {
        uint64_t best = UINT64_MAX;
        uint32_t bp = 0;
        for (uint32_t p = 0; p < n_parts; ++p) {
            const uint64_t v = pos[p] < k ? parts[((uint64_t)p * N + i) * k + pos[p]] : UINT64_MAX;
            if (v < best) {
                best = v;
                bp = p;
            }
        }
        if (best != UINT64_MAX) pos[bp]++;
        out[(uint64_t)i * k + s] = best;
    }
}

int nmz_knn_merge_dev(nmz_ctx *ctx, const uint64_t *d_parts, uint32_t n_parts, uint32_t n_traces, uint32_t k,
                      uint64_t *d_out, void *stream) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_parts >= 1 && n_parts <= 8, "n_parts must be in [1, 8]");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0 || k == 0) return NMZ_OK;
    hipLaunchKernelGGL(k_knn_merge, dim3(ceil_div(n_traces, 256)), dim3(256), 0,
                       stream ? (hipStream_t)stream : ctx->stream, d_parts, n_parts, n_traces, k, d_out);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

int nmz_ed_knn_fill_dev(nmz_ed_plan *plan, uint32_t k, uint64_t *d_knn_keys, void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    NMZ_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    if (plan->n == 0) return NMZ_OK;
    NMZ_CHECK(d_knn_keys != nullptr, "d_knn_keys is NULL");
    hipLaunchKernelGGL(k_knn_fill, dim3(ceil_div(plan->n, 256)), dim3(256), 0,
                       stream ? (hipStream_t)stream : plan->ctx->stream, d_knn_keys, plan->n, k, plan->n,
                       plan->band + 1, 1);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

int nmz_ed_allpairs_knn(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t n_traces, uint32_t band,
                        uint32_t k, uint32_t *knn_id, uint32_t *knn_dist) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(k <= 64, "k must be <= 64");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0 || k == 0) return NMZ_OK;
    nmz_ed_plan *plan = nullptr;
    NMZ_TRY(ed_plan_build(ctx, off, sym, n_traces, band, &plan));
    struct G {
        nmz_ed_plan *p;
        ~G() {
            p->mem.release();
            p->tp_mem.release();
            p->tp_ent.release();
            p->tp_rec.release();
            for (auto &kv : p->tile_list) kv.second.release();
            ed_tp_flag_release(p);
            delete p;
        }
    } pg{plan};
    hipStream_t st = ctx->stream;
    const uint64_t nk = (uint64_t)n_traces * k;
    NMZ_TRY(ctx->buf[2].ensure(Carve::bytes_for(nk, 8) + Carve::bytes_for(nk, 4) * 2));
    Carve cv(ctx->buf[2].ptr);
    uint64_t *d_knn = cv.take<uint64_t>(nk);
    uint32_t *d_id = cv.take<uint32_t>(nk);
    uint32_t *d_ds = cv.take<uint32_t>(nk);
    NMZ_TRY(ed_knn_run(plan, st, k, d_knn));
    hipLaunchKernelGGL(k_knn_final, dim3(ceil_div(nk, 256)), dim3(256), 0, st, d_knn, nk, d_id, d_ds);
    NMZ_HIP(hipGetLastError());
    if (knn_id) NMZ_HIP(hipMemcpyAsync(knn_id, d_id, nk * 4, hipMemcpyDeviceToHost, st));
    if (knn_dist) NMZ_HIP(hipMemcpyAsync(knn_dist, d_ds, nk * 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_ed_pairs(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t n_traces, const uint32_t *pairs,
                 uint64_t n_pairs, uint32_t band, uint32_t *dist) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(band < (1u << 20), "band too large");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_pairs == 0) return NMZ_OK;
    NMZ_CHECK(pairs && dist && off, "NULL argument");
    for (uint64_t t = 0; t < 2 * n_pairs; ++t) NMZ_CHECK(pairs[t] < n_traces, "pair index out of range");
    hipStream_t st = ctx->stream;
    const uint64_t total = n_traces ? off[n_traces] : 0;
    const unsigned gthreads = (unsigned)std::min<uint64_t>(256 * 1024, (n_pairs + 255) / 256 * 256);
    NMZ_TRY(ctx->buf[4].ensure(Carve::bytes_for(n_traces + 1, 8) + Carve::bytes_for(total + 1, 8) +
                               Carve::bytes_for(2 * n_pairs, 4) + Carve::bytes_for(n_pairs, 4) +
                               Carve::bytes_for((uint64_t)(2 * band + 1) * gthreads, 4)));
    Carve cv(ctx->buf[4].ptr);
    uint64_t *d_off = cv.take<uint64_t>(n_traces + 1);
    uint64_t *d_sym = cv.take<uint64_t>(total + 1);
    uint32_t *d_pairs = cv.take<uint32_t>(2 * n_pairs);
    uint32_t *d_dist = cv.take<uint32_t>(n_pairs);
    uint32_t *d_row = cv.take<uint32_t>((uint64_t)(2 * band + 1) * gthreads);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (n_traces + 1) * 8, hipMemcpyHostToDevice, st));
    if (total) NMZ_HIP(hipMemcpyAsync(d_sym, sym, total * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_pairs, pairs, 2 * n_pairs * 4, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_ed_generic, dim3(gthreads / 256), dim3(256), 0, st, d_off, d_sym, d_pairs, n_pairs, band, d_row,
                       d_dist);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipMemcpyAsync(dist, d_dist, n_pairs * 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

}  // extern "C"
