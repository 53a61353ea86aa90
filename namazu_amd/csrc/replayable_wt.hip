// K1 -- replayable-policy seed sweep statistics from wavelet trees (replayablepolicy.go:100-114).
//
// What a sweep returns per seed is the statistics of its E decisions t_e = FNV1a64(seed || hint_e) % m:
// the sum, the maximum and the first event index of the maximum. replayable.hip explains the algebra this
// starts from: per (table row L, hint-length class) segment of n events, sorted by the FNV correction C,
//     t_i = (b_i + Cm_i) mod m,   b_i = Hm for i < d (carry-free prefix), Hm2 for i >= d,
// where d = #{C_i <= ~H} and every t wraps at most once. So per (seed, segment)
//     sum  = d Hm + (n - d) Hm2 + sum Cm - m W,   W = #{i < d: Cm_i >= m - Hm} + #{i >= d: Cm_i >= m - Hm2}
//     max  = over the two parts, b + (the largest Cm below m - b), or, when no Cm of the part is below m - b,
//            b + (the part's largest Cm) - m.
// Both are 2-D dominance queries over the points (position i, rank of (Cm_i, ~e_i)). The plan stores, per
// (row, segment), a levelwise wavelet tree over the rank permutation in position order; a query answers
// "how many of positions < d have rank >= R" in one read per level, and the same descent finds the level
// where the predecessor of R inside the part branches off, from which a short second descent reaches it.
// Ranks sort by (Cm ascending, e descending), so among equal Cm the highest rank is the first event: the
// predecessor's event is the reference's first-index argmax (the order of its `>` test).
//
// Per (seed, segment of n ~ 2,000 events): ~3 lifting searches of ~5 LDS reads (d over C's high words,
// R_A and R_B over the sorted Cm through 256-bucket indexes), 2 x ceil(log2 n + 1) descent reads, a few
// predecessor reads -- ~50 LDS reads instead of ~150 for the sorted-block searches of k_replayable_sweep_oq,
// and a row image of ~13 B per event instead of ~27, so two rows fit one CU's LDS.
#include <algorithm>
#include <cstring>
#include <numeric>
#include <cstdlib>
#include <string>
#include <vector>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

#ifndef NMZ_WT_BRUTE
#define NMZ_WT_BRUTE 8
#endif
// segments of at most this many events: per-event decisions (32, for configs[1]'s 25-event segment: K1 0.062 ->
// 0.0675 ms, profiles/r05/k1/brute_ab)
constexpr uint32_t WT_BRUTE = NMZ_WT_BRUTE;
constexpr uint32_t WT_NMAX = 4096;     // largest segment the plan kernel sorts in LDS
constexpr uint32_t WT_LDS_MAX = 160 * 1024 - 256;  // dynamic LDS; the sweep kernel's few static bytes need the rest
constexpr uint32_t WT_NONE = 0xffffffffu;
constexpr uint32_t WT_PAD = 32;
#ifdef WT_BUILD_TRACE
// timing-only builds: wall_clock64() at the plan kernel's phase boundaries, per workgroup (tools/wt_build_trace.py)
constexpr uint32_t WT_TRACE_PHASES = 10, WT_TRACE_WGS = 8192;
__device__ unsigned long long g_wt_build_trace[WT_TRACE_WGS * WT_TRACE_PHASES];
#define WT_STAMP(k)                                                                                              \
    do {                                                                                                         \
        if (threadIdx.x == 0 && blockIdx.y * gridDim.x + blockIdx.x < WT_TRACE_WGS)                              \
            g_wt_build_trace[(L * gridDim.x + c) * WT_TRACE_PHASES + (k)] = wall_clock64();                      \
    } while (0)
#else
#define WT_STAMP(k) \
    do {            \
    } while (0)
#endif        // sentinels past Cm and C_hi: lifting searches of <= 5 rounds need no clamp

// WtClass (the segment descriptor) is in nmz_internal.h: the plan's host code packs it with the plan's inputs

// The tree stores the levels above the rank blocks of 2^bb ranks (bb = 5, 6 or 7: 32-, 64- or 128-rank blocks, the
// plan's choice, wt_layout); the blocks' prefix masks stand for the last bb levels. A wider block takes levels off
// both descents (each level one dependent LDS read per chain) for a larger image: ~2^bb / 8 bytes of masks per
// event (4, 8, 16). configs[1] (profiles/r05/k1/blocks_ab): bb = 6 takes K1 0.0656 -> 0.0623 ms and the pipelined
// step 0.0721 -> 0.0712 ms (84 KB images); bb = 7 (118 KB) runs K1 at 0.066 ms (its 128-bit mask arithmetic) and
// leaves the step's other kernels too little LDS beside it (step 0.082 ms), so plans take at most bb = 6.
__host__ __device__ constexpr uint32_t wt_levels(uint32_t K, uint32_t bb) { return K > bb ? K - bb : 0; }
// block masks' bytes: (n >> bb) + 1 blocks of 2^bb + 1 prefix masks of 2^bb bits
__host__ __device__ constexpr uint64_t wt_mask_bytes(uint32_t n, uint32_t bb) {
    return (uint64_t)((n >> bb) + 1) * ((1u << bb) + 1) * ((1u << bb) / 8);
}

// A block's prefix mask (2^BB bits) and the few operations the descents need on it
template <int BB>
struct WtMask;
template <>
struct WtMask<5> {
    using T = uint32_t;
    static __device__ __forceinline__ T load(const char *mk, uint32_t i) {
        return reinterpret_cast<const uint32_t *>(mk)[i];
    }
    static __device__ __forceinline__ uint32_t count_ge(T v, uint32_t r) { return __popc(v >> r); }  // bits >= r
    static __device__ __forceinline__ T below(T v, uint32_t r) { return __builtin_amdgcn_ubfe(v, 0u, r); }  // r < 32
    static __device__ __forceinline__ T low(T v, uint32_t s) { return v & (0xffffffffu >> (32u - s)); }  // 1..32
    static __device__ __forceinline__ T inv(T v) { return ~v; }
    static __device__ __forceinline__ bool any(T v) { return v != 0; }
    static __device__ __forceinline__ uint32_t top(T v) { return 31u - __clz(v); }  // v != 0
};
template <>
struct WtMask<6> {
    using T = uint64_t;
    static __device__ __forceinline__ T load(const char *mk, uint32_t i) {
        return reinterpret_cast<const uint64_t *>(mk)[i];
    }
    static __device__ __forceinline__ uint32_t count_ge(T v, uint32_t r) { return (uint32_t)__popcll(v >> r); }
    static __device__ __forceinline__ T below(T v, uint32_t r) { return v & ((1ull << r) - 1ull); }
    static __device__ __forceinline__ T low(T v, uint32_t s) { return v & (~0ull >> (64u - s)); }
    static __device__ __forceinline__ T inv(T v) { return ~v; }
    static __device__ __forceinline__ bool any(T v) { return v != 0; }
    static __device__ __forceinline__ uint32_t top(T v) { return 63u - (uint32_t)__clzll(v); }
};
struct WtMask128 {
    uint64_t lo, hi;
};
template <>
struct WtMask<7> {
    using T = WtMask128;
    static __device__ __forceinline__ T load(const char *mk, uint32_t i) {
        const uint4 x = reinterpret_cast<const uint4 *>(mk)[i];
        return T{((uint64_t)x.y << 32) | x.x, ((uint64_t)x.w << 32) | x.z};
    }
    static __device__ __forceinline__ uint32_t count_ge(T v, uint32_t r) {
        return r < 64 ? (uint32_t)(__popcll(v.lo >> r) + __popcll(v.hi)) : (uint32_t)__popcll(v.hi >> (r - 64));
    }
    static __device__ __forceinline__ T below(T v, uint32_t r) {
        return r < 64 ? T{v.lo & ((1ull << r) - 1ull), 0ull} : T{v.lo, v.hi & ((1ull << (r - 64)) - 1ull)};
    }
    static __device__ __forceinline__ T low(T v, uint32_t s) {
        return s <= 64 ? T{v.lo & (~0ull >> (64u - s)), 0ull} : T{v.lo, v.hi & (~0ull >> (128u - s))};
    }
    static __device__ __forceinline__ T inv(T v) { return T{~v.lo, ~v.hi}; }
    static __device__ __forceinline__ bool any(T v) { return (v.lo | v.hi) != 0; }
    static __device__ __forceinline__ uint32_t top(T v) {
        return v.hi ? 127u - (uint32_t)__clzll(v.hi) : 63u - (uint32_t)__clzll(v.lo);
    }
};

// ---------------------------------------------------------------------------------------------------------------
// plan: one workgroup per (segment, row L). Sorts the segment's keys (Cm << 32 | (0xffff - e) << 16 | position)
// in LDS (bitonic), writes Cm / e by rank and C_hi by position, the two bucket indexes, and the K wavelet levels:
// level l holds bit K-1-l of the ranks, in the order "stably sorted by the top l bits" (the node of the value
// prefix pi starts at pi << (K-l), since the ranks are a permutation of [0, n)), one {32 bits, ones before} pair
// per 32 positions. Also adds the segment's sum of Cm to the row sum (every segment, short ones included).
// ---------------------------------------------------------------------------------------------------------------
constexpr uint32_t WT_BT = 512, WT_BW = WT_BT / 64;  // plan kernel: threads and waves per workgroup

// exclusive scan in place over nb <= 2,048 bucket counts (4 per thread, wave scans, then the wave totals in cum);
// *big gets the largest count above 32 (a bucket the per-bucket insertion sort should not take)
__device__ __forceinline__ void wt_bucket_scan(uint32_t *bc, uint32_t nb, uint32_t *cum, uint32_t *big, uint32_t tid) {
    const uint32_t lane = tid & 63, wave = tid >> 6, b0 = 4 * tid;
    uint32_t c4[4], t = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        c4[k] = b0 + k < nb ? bc[b0 + k] : 0u;
        t += c4[k];
        if (c4[k] > 32) atomicMax(big, c4[k]);
    }
    uint32_t inc = t;
    for (int o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(inc, o, 64);
        if (lane >= (uint32_t)o) inc += v;
    }
    if (lane == 63) cum[wave] = inc;
    __syncthreads();
    uint32_t base = inc - t;
    for (uint32_t w = 0; w < wave; ++w) base += cum[w];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        if (b0 + k < nb) bc[b0 + k] = base;  // bucket start (a cursor while scattering, then the end)
        base += c4[k];
    }
    __syncthreads();
}

// the plan's hints on the device, for the fused plan kernel (it computes and C-sorts its own table segments)
struct WtHints {
    const uint32_t *hoff;   // [E + 1] hint byte offsets (original event order)
    const uint8_t *hbytes;
    const uint32_t *perm;   // [E] length-sorted position -> event
    uint64_t m;             // the modulus (< 2^32 on this path) and floor(2^64 / m)
    uint64_t mu;
    uint4 *table;           // [256][E] out: {C lo, C hi, C mod m, ~e}, C-sorted per segment
    uint32_t *zero0;        // ranges the first workgroup zeroes (the plan's seed-scratch counters)
    uint32_t n_zero0;
    uint32_t *zero1;
    uint32_t n_zero1;
};

template <bool FUSED, int BB>
__global__ __launch_bounds__(WT_BT) void k_replayable_wt_build(const uint4 *__restrict__ table, uint32_t E,
                                                               WtClass *__restrict__ classes, uint32_t msh,
                                                               uint32_t mbits, uint4 *__restrict__ blob, uint32_t rb16,
                                                               unsigned long long *__restrict__ rowsum, WtHints hz) {
    // LDS (~73 KB, two workgroups per CU): the keys, then (after the sort) the rank arrays in their place; the
    // sorted keys; bucket counts (np / 2 buckets); level words and counts; small scratch
    extern __shared__ uint4 wt_build_lds[];
    uint64_t *key = reinterpret_cast<uint64_t *>(wt_build_lds);                 // [WT_NMAX]
    uint16_t *S0 = reinterpret_cast<uint16_t *>(key);                           // [2][WT_NMAX], after the sort
    uint64_t *srt = key + WT_NMAX;                                              // [WT_NMAX] sorted keys
    uint32_t *bc = reinterpret_cast<uint32_t *>(srt + WT_NMAX);                 // [WT_NMAX / 2]
    uint32_t *wb = bc + WT_NMAX / 2;                                            // [WT_NMAX / 32 + 4]
    uint32_t *cum = wb + WT_NMAX / 32 + 4;                                      // [WT_NMAX / 32 + 4]
    uint32_t *idx = cum + WT_NMAX / 32 + 4;                                     // [2][260] bucket indexes
    unsigned long long *part = reinterpret_cast<unsigned long long *>(idx + 520);  // [WT_BW]
    uint32_t *bmax = reinterpret_cast<uint32_t *>(part + WT_BW);               // [4]
    // workgroups start in dispatch order (x fastest): the largest segments' rows first, so the small segments'
    // short workgroups fill in behind them instead of holding slots the large ones wait for
    const uint32_t lin = blockIdx.y * gridDim.x + blockIdx.x, L = lin & 255u;
    const uint32_t c = classes[lin >> 8].order, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    WT_STAMP(0);
    const WtClass ci = classes[c];
    const uint32_t n = ci.n;
    uint32_t np = 1, lgp = 0;
    while (np < n) {
        np <<= 1;
        ++lgp;
    }
    const uint32_t nb = np >= 2 ? np / 2 : 1, lgb = lgp ? lgp - 1 : 0;  // sort buckets (~2 keys each) and their bits
    if (tid < 4) bmax[tid] = 0;
    char *img = reinterpret_cast<char *>(blob + (uint64_t)L * rb16);
    // the segment's entries, one load each (every load in flight): the row sum, C's high words and the sort keys
    constexpr uint32_t PPT = WT_NMAX / WT_BT;
    uint4 q[PPT];
    if constexpr (FUSED) {
        if (lin == 0) {
            for (uint32_t i = tid; i < hz.n_zero0; i += WT_BT) hz.zero0[i] = 0;
            for (uint32_t i = tid; i < hz.n_zero1; i += WT_BT) hz.zero1[i] = 0;
        }
        // C = FNV-1a(seed bytes L, hint) - L * P^len (the table's correction, k_replayable_table) for the segment's
        // events, a thread per event and all of a thread's events in step (one hint length per segment), then
        // the stable C order through LDS: a counting sort on C's top bits and an insertion sort per bucket, or a
        // bitonic sort of (C, position) when a bucket holds more than 32 (repeated hints)
        uint16_t *posL = reinterpret_cast<uint16_t *>(key);  // [WT_NMAX] the sorted order's positions
        uint16_t *eL = posL + WT_NMAX;                       // [WT_NMAX] event by position (E <= 65,536)
        uint64_t h[PPT];
        uint32_t b0[PPT];
        uint32_t len = 0;
#pragma unroll
        for (uint32_t k = 0; k < PPT; ++k) {
            const uint32_t i = tid + k * WT_BT;
            h[k] = L;
            b0[k] = 0;
            if (i < n) {
                const uint32_t e = hz.perm[ci.start + i];
                eL[i] = (uint16_t)e;
                b0[k] = hz.hoff[e];
                len = hz.hoff[e + 1] - b0[k];
            }
        }
        len = __builtin_amdgcn_readfirstlane(len);  // lane 0 holds an event of the segment (n >= 1)
        // 16 hint bytes per round: the 5 aligned words covering them, all rounds' loads in flight together, then
        // v_alignbit to the hint's own byte order
        const uint32_t *__restrict__ hw = reinterpret_cast<const uint32_t *>(hz.hbytes);
        for (uint32_t c0 = 0; c0 < len; c0 += 16) {
            uint32_t w[PPT][5];
#pragma unroll
            for (uint32_t k = 0; k < PPT; ++k) {
                const uint32_t a = (b0[k] + c0) >> 2, wl = (b0[k] + len - 1) >> 2;
#pragma unroll
                for (uint32_t j = 0; j < 5; ++j) w[k][j] = tid + k * WT_BT < n ? hw[min(a + j, wl)] : 0u;
            }
#pragma unroll
            for (uint32_t k = 0; k < PPT; ++k) {
                const uint32_t sh = 8 * (b0[k] & 3);
                uint32_t u[4];
#pragma unroll
                for (uint32_t j = 0; j < 4; ++j) u[j] = __builtin_amdgcn_alignbit(w[k][j + 1], w[k][j], sh);
#pragma unroll
                for (uint32_t b = 0; b < 16; ++b)
                    if (c0 + b < len) h[k] = fnv_step(h[k], (u[b >> 2] >> (8 * (b & 3))) & 0xffu);
            }
        }
        const uint32_t shc = 64 - lgb;
        auto cb = [&](uint64_t C) { return lgb ? (uint32_t)(C >> shc) : 0u; };
        for (uint32_t b = tid; b < nb; b += WT_BT) bc[b] = 0;
        __syncthreads();
#pragma unroll
        for (uint32_t k = 0; k < PPT; ++k) {
            h[k] -= (uint64_t)L * ci.pn;  // C
            if (tid + k * WT_BT < n) atomicAdd(&bc[cb(h[k])], 1u);
        }
        __syncthreads();
        wt_bucket_scan(bc, nb, cum, bmax + 1, tid);
        if (bmax[1] == 0) {
#pragma unroll
            for (uint32_t k = 0; k < PPT; ++k) {
                const uint32_t i = tid + k * WT_BT;
                if (i < n) {
                    const uint32_t slot = atomicAdd(&bc[cb(h[k])], 1u);
                    srt[slot] = h[k];
                    posL[slot] = (uint16_t)i;
                }
            }
            __syncthreads();
            for (uint32_t b = tid; b < nb; b += WT_BT) {  // bucket b: [end of b - 1, end of b)
                const uint32_t lo = b ? bc[b - 1] : 0u, hi = bc[b];
                for (uint32_t i = lo + 1; i < hi; ++i) {
                    const uint64_t v = srt[i];
                    const uint16_t pv = posL[i];
                    uint32_t j = i;
                    while (j > lo && (srt[j - 1] > v || (srt[j - 1] == v && posL[j - 1] > pv))) {
                        srt[j] = srt[j - 1];
                        posL[j] = posL[j - 1];
                        --j;
                    }
                    srt[j] = v;
                    posL[j] = pv;
                }
            }
        } else {
#pragma unroll
            for (uint32_t k = 0; k < PPT; ++k) {
                const uint32_t i = tid + k * WT_BT;
                if (i < np) {
                    srt[i] = i < n ? h[k] : ~0ull;
                    posL[i] = (uint16_t)i;
                }
            }
            for (uint32_t k = 2; k <= np; k <<= 1)
                for (uint32_t j = k >> 1; j; j >>= 1) {
                    __syncthreads();
                    for (uint32_t i = tid; i < np; i += WT_BT) {
                        const uint32_t l = i ^ j;
                        if (l > i) {
                            const uint64_t a = srt[i], b = srt[l];
                            const uint16_t pa = posL[i], pb = posL[l];
                            if ((a > b || (a == b && pa > pb)) == ((i & k) == 0)) {
                                srt[i] = b;
                                srt[l] = a;
                                posL[i] = pb;
                                posL[l] = pa;
                            }
                        }
                    }
                }
        }
        __syncthreads();
        // the C-sorted entries (thread tid holds positions tid + k * WT_BT), written out as the table's row segment
        uint4 *__restrict__ out = hz.table + (uint64_t)L * E + ci.start;
#pragma unroll
        for (uint32_t k = 0; k < PPT; ++k) {
            const uint32_t j = tid + k * WT_BT;
            q[k] = make_uint4(0, 0, 0, 0);
            if (j < n) {
                const uint64_t C = srt[j];
                const uint32_t e = eL[posL[j]];
                q[k] = make_uint4((uint32_t)C, (uint32_t)(C >> 32), mod_barrett64(C, hz.m, hz.mu), ~e);
                out[j] = q[k];
            }
        }
        __syncthreads();  // posL (the key region) and srt are free again
    } else {
        const uint4 *__restrict__ row = table + (uint64_t)L * E + ci.start;
#pragma unroll
        for (uint32_t k = 0; k < PPT; ++k) {
            const uint32_t i = tid + k * WT_BT;
            q[k] = i < n ? row[i] : make_uint4(0, 0, 0, 0);
        }
    }
    uint64_t s = 0;
#pragma unroll
    for (uint32_t k = 0; k < PPT; ++k) s += q[k].z;
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) part[wave] = s;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (uint32_t w = 0; w < WT_BW; ++w) t += part[w];
        atomicAdd(rowsum + L, t);
    }
    WT_STAMP(1);
    if (n <= WT_BRUTE) return;
    uint32_t *chi_img = reinterpret_cast<uint32_t *>(img + ci.o_chi);
#pragma unroll
    for (uint32_t k = 0; k < PPT; ++k) {
        const uint32_t i = tid + k * WT_BT;
        if (i >= n) break;
        chi_img[i] = q[k].y;
        const uint32_t e = ~q[k].w;  // < 65536 (the host checks E)
        key[i] = ((uint64_t)q[k].z << 32) | ((uint64_t)(0xffffu - e) << 16) | i;
    }
    WT_STAMP(2);
    // sort the keys: counting sort on the top lg(np) - 1 bits of Cm (uniform in [0, m): ~2 keys per bucket), then an
    // insertion sort per bucket (a thread per bucket); a bucket of more than 32 keys (repeated hints: equal Cm)
    // sends the whole segment to a bitonic sort
    {
        const uint32_t sh = mbits > lgb ? mbits - lgb : 0u;
        for (uint32_t b = tid; b < nb; b += WT_BT) bc[b] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += WT_BT) atomicAdd(&bc[(uint32_t)(key[i] >> 32) >> sh], 1u);
        __syncthreads();
        wt_bucket_scan(bc, nb, cum, bmax, tid);
        if (bmax[0] <= 32) {
            for (uint32_t i = tid; i < n; i += WT_BT) {
                const uint64_t kk = key[i];
                srt[atomicAdd(&bc[(uint32_t)(kk >> 32) >> sh], 1u)] = kk;
            }
            __syncthreads();
            for (uint32_t b = tid; b < nb; b += WT_BT) {  // bucket b: [end of b - 1, end of b)
                const uint32_t lo = b ? bc[b - 1] : 0u, hi = bc[b];
                for (uint32_t i = lo + 1; i < hi; ++i) {
                    const uint64_t v = srt[i];
                    uint32_t j = i;
                    while (j > lo && srt[j - 1] > v) {
                        srt[j] = srt[j - 1];
                        --j;
                    }
                    srt[j] = v;
                }
            }
        } else {
            for (uint32_t i = n + tid; i < np; i += WT_BT) key[i] = ~0ull;
            for (uint32_t k = 2; k <= np; k <<= 1)
                for (uint32_t j = k >> 1; j; j >>= 1) {
                    __syncthreads();
                    for (uint32_t i = tid; i < np; i += WT_BT) {
                        const uint32_t l = i ^ j;
                        if (l > i) {
                            const uint64_t a = key[i], b = key[l];
                            if ((a > b) == ((i & k) == 0)) {
                                key[i] = b;
                                key[l] = a;
                            }
                        }
                    }
                }
            __syncthreads();
            for (uint32_t i = tid; i < n; i += WT_BT) srt[i] = key[i];
        }
        __syncthreads();  // the keys' region becomes the rank arrays
        WT_STAMP(3);
    }
    uint32_t *chiL = reinterpret_cast<uint32_t *>(key) + WT_NMAX;  // C_hi by position (the bucket index below)
#pragma unroll
    for (uint32_t k = 0; k < PPT; ++k) {
        const uint32_t i = tid + k * WT_BT;
        if (i < n) chiL[i] = q[k].y;
    }
    uint32_t *cm_img = reinterpret_cast<uint32_t *>(img + ci.o_cm);
    uint16_t *e_img = reinterpret_cast<uint16_t *>(img + ci.o_e);
    for (uint32_t j = tid; j < n; j += WT_BT) {
        const uint64_t kk = srt[j];
        cm_img[j] = (uint32_t)(kk >> 32);
        e_img[j] = (uint16_t)(0xffffu - ((kk >> 16) & 0xffffu));
        S0[kk & 0xffffu] = (uint16_t)j;
    }
    if (tid < WT_PAD) {
        cm_img[n + tid] = ~0u;  // sentinels: never below a search bound
        chi_img[n + tid] = ~0u;
    }
    __syncthreads();  // chiL complete
    WT_STAMP(4);
    // bucket indexes (first rank with Cm >= b << msh, b <= 256; first position with C_hi >= b << 24, b < 256): every
    // position writes the buckets between its predecessor's and its own (the sorted order's boundaries)
    uint32_t *im = idx, *ic = idx + 260;
    for (uint32_t i = tid; i <= n; i += WT_BT) {
        const int bm = i < n ? (int)((uint32_t)(srt[i] >> 32) >> msh) : 257;
        const int pm_ = i ? (int)((uint32_t)(srt[i - 1] >> 32) >> msh) : -1;
        for (int b = pm_ + 1; b <= min(bm, 256); ++b) im[b] = i;
        const int bc2 = i < n ? (int)(chiL[i] >> 24) : 256;
        const int pc = i ? (int)(chiL[i - 1] >> 24) : -1;
        for (int b = pc + 1; b <= min(bc2, 255); ++b) ic[b] = i;
    }
    __syncthreads();
    if (tid < 257) {
        reinterpret_cast<uint16_t *>(img + ci.o_im)[tid] = (uint16_t)im[tid];
        atomicMax(bmax + 2, (tid < 256 ? im[tid + 1] : n) - im[tid]);
    }
    if (tid < 256) {
        reinterpret_cast<uint16_t *>(img + ci.o_ic)[tid] = (uint16_t)ic[tid];
        atomicMax(bmax + 3, (tid < 255 ? ic[tid + 1] : n) - ic[tid]);
    }
    __syncthreads();
#ifndef WT_ABL_RS_ATOMIC
    if (tid == 0) atomicMax(&classes[c].rS, 32u - __clz(max(bmax[2], bmax[3])));
#endif
    WT_STAMP(5);
    WT_STAMP(6);
    // wavelet levels above the 32-rank blocks. Per level, wave w ballots a contiguous range of 64-position groups
    // (bit K-1-l of the rank at each position, in this level's order), the 8 wave totals give each wave its ones
    // before its range, and every position's destination in the next level's order follows from the ones before it
    // in its node: one barrier for the totals, one for the next order (no serial scan of the words).
    const uint32_t K = ci.K, nw = ci.nw, lb = wt_levels(K, BB);
    uint2 *lv = reinterpret_cast<uint2 *>(img + ci.o_lv);
    uint16_t *cur = S0, *nxt = S0 + WT_NMAX;
    constexpr uint32_t MAXG = (WT_NMAX / 64 + 1 + WT_BW - 1) / WT_BW;  // groups per wave, at most
    const uint32_t ng = (nw * 32 + 63) / 64, gpw = (ng + WT_BW - 1) / WT_BW, g0 = wave * gpw;
    uint32_t *wtot = cum;  // [WT_BW]
    for (uint32_t l = 0; l < lb; ++l) {
        const uint32_t h = 1u << (K - l - 1);
        uint64_t bal[MAXG];
        uint32_t vv[MAXG], tot = 0;
#pragma unroll
        for (uint32_t gi = 0; gi < MAXG; ++gi) {
            const uint32_t g = g0 + gi, j = g * 64 + lane;
            bal[gi] = 0;
            vv[gi] = 0;
            if (gi < gpw && g < ng) {
                vv[gi] = j < n ? cur[j] : 0u;
                bal[gi] = __ballot(j < n && (vv[gi] & h));
                tot += (uint32_t)__popcll(bal[gi]);
            }
        }
        if (lane == 0) wtot[wave] = tot;
        __syncthreads();
        uint32_t pre = 0;
        for (uint32_t w = 0; w < wave; ++w) pre += wtot[w];
        const uint64_t below = (1ull << lane) - 1ull;
#pragma unroll
        for (uint32_t gi = 0; gi < MAXG; ++gi) {
            const uint32_t g = g0 + gi, j = g * 64 + lane;
            if (gi < gpw && g < ng) {
                const uint64_t bg = bal[gi];
                if (lane == 0) lv[l * nw + 2 * g] = make_uint2((uint32_t)bg, pre);
                if (lane == 1 && 2 * g + 1 < nw)
                    lv[l * nw + 2 * g + 1] = make_uint2((uint32_t)(bg >> 32), pre + (uint32_t)__popc((uint32_t)bg));
                if (j < n) {
                    const uint32_t v = vv[gi];
                    const uint32_t s0 = v & ~(2 * h - 1);  // the node's first position
                    const uint32_t r1 = pre + (uint32_t)__popcll(bg & below) - (s0 >> 1);
                    nxt[(v & h) ? s0 + h + r1 : j - r1] = (uint16_t)v;
                }
                pre += (uint32_t)__popcll(bg);
            }
        }
        __syncthreads();
        uint16_t *t = cur;
        cur = nxt;
        nxt = t;
    }
    WT_STAMP(7);
    // level lb: the node of block b holds the ranks [2^BB b, 2^BB (b + 1)) in position order (all n ranks when K <= BB);
    // entry o of block b = the OR of bit (rank mod 2^BB) over the block's first o entries: a prefix OR per block
    const uint32_t nbk = (n >> BB) + 1;
    if constexpr (BB == 5) {  // two blocks per wave step, 32 lanes each
        uint32_t *mk = reinterpret_cast<uint32_t *>(img + ci.o_mk);
        for (uint32_t b0 = 2 * wave; b0 < nbk; b0 += 2 * WT_BW) {
            const uint32_t b = b0 + (lane >> 5), j = 32 * b + (lane & 31);
            uint32_t v = (b < nbk && j < n) ? 1u << (cur[j] & 31) : 0u;
            for (int o = 1; o < 32; o <<= 1) {
                const uint32_t u = __shfl_up(v, o, 64);
                if ((lane & 31) >= (uint32_t)o) v |= u;
            }
            if (b < nbk) {
                mk[b * 33 + (lane & 31) + 1] = v;
                if ((lane & 31) == 0) mk[b * 33] = 0;
            }
        }
    } else if constexpr (BB == 6) {  // a block per wave step
        uint64_t *mk = reinterpret_cast<uint64_t *>(img + ci.o_mk);
        for (uint32_t b = wave; b < nbk; b += WT_BW) {
            const uint32_t j = 64 * b + lane;
            unsigned long long v = j < n ? 1ull << (cur[j] & 63) : 0ull;
            for (int o = 1; o < 64; o <<= 1) {
                const unsigned long long u = __shfl_up(v, o, 64);
                if (lane >= (uint32_t)o) v |= u;
            }
            mk[b * 65 + lane + 1] = v;
            if (lane == 0) mk[b * 65] = 0;
        }
    } else {  // a block per wave step, in two halves of 64 entries (the second half ORs in the first's total)
        uint4 *mk = reinterpret_cast<uint4 *>(img + ci.o_mk);
        for (uint32_t b = wave; b < nbk; b += WT_BW) {
            unsigned long long clo = 0, chi = 0;
            for (uint32_t hf = 0; hf < 2; ++hf) {
                const uint32_t j = 128 * b + 64 * hf + lane, r = j < n ? (uint32_t)(cur[j] & 127) : 0u;
                unsigned long long lo = (j < n && r < 64) ? 1ull << r : 0ull;
                unsigned long long hi = (j < n && r >= 64) ? 1ull << (r - 64) : 0ull;
                for (int o = 1; o < 64; o <<= 1) {
                    const unsigned long long ul = __shfl_up(lo, o, 64), uh = __shfl_up(hi, o, 64);
                    if (lane >= (uint32_t)o) {
                        lo |= ul;
                        hi |= uh;
                    }
                }
                lo |= clo;
                hi |= chi;
                mk[b * 129 + 64 * hf + lane + 1] =
                    make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
                clo = __shfl(lo, 63, 64);
                chi = __shfl(hi, 63, 64);
            }
            if (lane == 0) mk[b * 129] = make_uint4(0u, 0u, 0u, 0u);
        }
    }
#ifdef WT_BUILD_TRACE
    __syncthreads();
#endif
    WT_STAMP(8);
}

// ---------------------------------------------------------------------------------------------------------------
// sweep
// ---------------------------------------------------------------------------------------------------------------
// one decision from a table entry {C lo, C hi, Cm, ~e}: counts carry-free events (d) and wraps (W).
// BIG: m >= 2^31, where base + Cm can overflow 32 bits (the true sum then exceeds m and t = sum - m is exact
// modulo 2^32)
template <bool BIG>
__device__ __forceinline__ void wt_decide(uint4 q, uint64_t nH, uint32_t Hm, uint32_t Hm2, uint32_t m, uint32_t &d,
                                          uint32_t &W, uint64_t &key) {
    const bool nc = (((uint64_t)q.y << 32) | q.x) <= nH;
    const uint32_t b = nc ? Hm : Hm2;
    const uint32_t s = b + q.z;
    const bool wrap = BIG ? (s < b || s >= m) : s >= m;
    const uint32_t t = wrap ? s - m : s;
    d += nc;
    W += wrap;
    const uint64_t k = ((uint64_t)t << 32) | q.w;
    key = k > key ? k : key;
}

// Wave-uniform operands of the descents copied into VGPRs, so their VOP2 forms take no SGPR or inline-constant
// operand (tools/ubench measures those forms at half the VGPR-only issue rate): 1-2 % on K1, consistently across
// four A/B pairs (profiles/r03r_wt_vgprc_ab.json); -DWT_SGPR_CONST builds the compiler's forms
#ifndef WT_SGPR_CONST
__device__ __forceinline__ uint32_t wt_v(uint32_t x) {
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}
#else
__device__ __forceinline__ uint32_t wt_v(uint32_t x) { return x; }
#endif

// ones among the first p entries of a level, minus those before the node that starts at s (s >> 1: every node
// before it is whole and half ones)
__device__ __forceinline__ uint32_t wt_ones(const uint2 *__restrict__ lvl, uint32_t s, uint32_t p) {
    const uint2 w = lvl[p >> 5];
    return w.y + __popc(w.x & ((1u << (p & 31)) - 1u)) - (s >> 1);
}


// One seed's statistics over one segment: adds d Hm + (n - d) Hm2 to sum, the segment's wraps to W, and folds its
// maximum key {t, ~e} into key.
// wave-uniform constants the sweep keeps in VGPRs (operands of VOP2 forms)
struct WtVConst {
    uint32_t st4[5];  // lifting-search steps in bytes: 4 << r
};

// NS seeds per lane (arrays indexed by u, unrolled): the wave-uniform control -- segment parameters, lifting
// rounds, level constants, loop trips, ballots -- is paid once for NS seeds, and the NS seeds' read chains are
// independent, so a wave keeps 2 NS dependent LDS chains in flight per descent level instead of 2.
template <bool BIG, int NS, int BB>
__device__ __forceinline__ void wt_seed_class(const WtVConst &vc, const WtClass &ci, const char *__restrict__ img,
                                              const uint4 *__restrict__ row, const uint64_t (&h0)[NS], uint32_t m,
                                              uint64_t mu, uint32_t m_k64, uint32_t msh, uint64_t (&sum)[NS],
                                              uint32_t (&W)[NS], uint64_t (&key)[NS]) {
    const uint32_t n = ci.n;
    uint64_t nH[NS];
    uint32_t Hm[NS], Hm2[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const uint64_t H = h0[u] * ci.pn;
        nH[u] = ~H;
        Hm[u] = BIG ? mod_barrett64(H, m, mu) : mod_barrett_small(H, m, mu);
        const uint32_t t2 = Hm[u] + m_k64;
        Hm2[u] = BIG ? ((t2 < Hm[u] || t2 >= m) ? t2 - m : t2) : min(t2, t2 - m);
    }
    if (n <= WT_BRUTE) {
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            uint32_t d = 0;
            for (uint32_t i = 0; i < n; ++i) wt_decide<BIG>(row[ci.start + i], nH[u], Hm[u], Hm2[u], m, d, W[u], key[u]);
            sum[u] += (uint64_t)d * Hm[u] + (uint64_t)(n - d) * Hm2[u];
        }
        return;
    }
    const uint32_t *__restrict__ cm = reinterpret_cast<const uint32_t *>(img + ci.o_cm);
    const uint32_t *__restrict__ chi = reinterpret_cast<const uint32_t *>(img + ci.o_chi);
    const uint16_t *__restrict__ ev = reinterpret_cast<const uint16_t *>(img + ci.o_e);
    const uint16_t *__restrict__ im = reinterpret_cast<const uint16_t *>(img + ci.o_im);
    const uint16_t *__restrict__ ic = reinterpret_cast<const uint16_t *>(img + ci.o_ic);
    uint32_t nh[NS], XA[NS], XB[NS];
    const uint32_t *pa[NS], *pb[NS], *pc[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        nh[u] = (uint32_t)(nH[u] >> 32);
        XA[u] = m - Hm[u];  // t wraps <=> Cm >= X
        XB[u] = m - Hm2[u];
        // three lifting searches stepped together (every read of a round in flight at once) from the bucket starts:
        // every entry past the bucket is >= the bound, and the sentinel at n ends every probe past the array
        // (pointer form: a round's probes are LDS reads with immediate offsets; WT_PAD sentinels end the probes of up
        // to five rounds past the array, longer searches -- repeated hints -- clamp at the sentinel at n)
        pa[u] = chi + ic[nh[u] >> 24];
        pb[u] = cm + im[XA[u] >> msh];
        pc[u] = cm + im[XB[u] >> msh];
    }
    const uint32_t rS = ci.rS;
#ifdef WT_ABL_LIFT
    if (0)
#endif
    if (rS <= 5) {
#pragma unroll
        for (int r = 4; r >= 0; --r) {
            if (rS > (uint32_t)r) {
                constexpr uint32_t one = 1;
                const uint32_t st = one << r, st4 = vc.st4[r];  // the step in bytes, in a VGPR (a VOP2 select)
#pragma unroll
                for (int u = 0; u < NS; ++u) {
                    const uint32_t a = pa[u][st - 1], b = pb[u][st - 1], c = pc[u][st - 1];
                    pa[u] = reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(pa[u]) + (a < nh[u] ? st4 : 0u));
                    pb[u] = reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(pb[u]) + (b < XA[u] ? st4 : 0u));
                    pc[u] = reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(pc[u]) + (c < XB[u] ? st4 : 0u));
                }
            }
        }
    } else {
        const uint32_t *ea = chi + n, *eb = cm + n;
        for (uint32_t st = (1u << rS) >> 1; st; st >>= 1) {
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const uint32_t a = *min(pa[u] + st - 1, ea), b = *min(pb[u] + st - 1, eb), c = *min(pc[u] + st - 1, eb);
                pa[u] += a < nh[u] ? st : 0u;
                pb[u] += b < XA[u] ? st : 0u;
                pc[u] += c < XB[u] ? st : 0u;
            }
        }
    }
    // (LDS addresses: the low words of the generic pointers)
    auto lo = [](const uint32_t *q) { return (uint32_t)reinterpret_cast<uintptr_t>(q); };
    uint32_t d[NS], RA[NS], RB[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        RA[u] = (lo(pb[u]) - lo(cm)) >> 2;
        RB[u] = (lo(pc[u]) - lo(cm)) >> 2;
        // d = #{C <= ~H}: #{C_hi < ~H_hi} plus the entries whose high word equals ~H_hi and low word is <= ~H_lo
        // (about n / 2^32 of the queries: the low words come from the table row)
        d[u] = (lo(pa[u]) - lo(chi)) >> 2;
        if (chi[d[u]] == nh[u]) {
            const uint32_t nl = (uint32_t)nH[u];
            while (d[u] < n && chi[d[u]] == nh[u] && row[ci.start + d[u]].x <= nl) ++d[u];
        }
    }
    // descents along R_A's and R_B's paths with the prefix [0, d) down to R's 32-rank block, branch-free with every
    // read of a level in flight: counts of ranks >= R, and the deepest level where a part's elements below R branch
    // off (the predecessor's subtree: node start s, prefix offset q)
    const uint2 *__restrict__ lv = reinterpret_cast<const uint2 *>(img + ci.o_lv);
    const char *__restrict__ mk = img + ci.o_mk;
    using MK = WtMask<BB>;
    using MT = typename MK::T;
    constexpr uint32_t BW = 1u << BB, BM = BW - 1;
#ifdef WT_ABL_COUNT
    const uint32_t K = ci.K, nw = ci.nw, lb = 0;
#else
    const uint32_t K = ci.K, nw = ci.nw, lb = wt_levels(K, BB);
#endif
    uint32_t oA[NS], oB[NS], cA[NS], cB[NS], lA[NS], sA[NS], qA[NS], lB[NS], sB[NS], qB[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        oA[u] = oB[u] = d[u];
        cA[u] = cB[u] = 0;
        lA[u] = lB[u] = WT_NONE;
        sA[u] = qA[u] = sB[u] = qB[u] = 0;
    }
    const uint32_t nv = wt_v(n), one = wt_v(1u), five = wt_v(5u);
    if (lb) {
        // level 0 (the root: both chains at offset d, one read); then the level constants live in VGPRs, halved per
        // level (no SGPR operands, no per-level scalar shifts)
        const uint32_t hs = 1u << (K - 1);
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const uint2 w = lv[d[u] >> 5];
            const uint32_t o = w.y + __popc(__builtin_amdgcn_ubfe(w.x, 0u, d[u])), z = d[u] - o;
            const bool b1 = RA[u] >= hs, b2 = RB[u] >= hs;
            const bool u1 = b1 && z != 0, u2 = b2 && hs > z;  // the root's left child is whole (n >= hs)
            lA[u] = u1 ? 1u : lA[u];
            qA[u] = u1 ? z : qA[u];
            lB[u] = u2 ? 1u : lB[u];
            qB[u] = u2 ? z : qB[u];
            cA[u] = b1 ? 0u : o;
            cB[u] = b2 ? 0u : o;
            oA[u] = b1 ? o : z;
            oB[u] = b2 ? o : z;
        }
        uint32_t h = wt_v(hs >> 1), msk = wt_v(~(hs - 1)), l1 = wt_v(2u);
        const uint2 *__restrict__ lvl = lv + nw;
        for (uint32_t l = 1; l < lb; ++l) {
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const uint32_t s1 = RA[u] & msk, p1 = s1 + oA[u], s2 = RB[u] & msk, p2 = s2 + oB[u];
                const uint2 w1 = lvl[p1 >> five], w2 = lvl[p2 >> five];
                const uint32_t o1 = w1.y + __popc(__builtin_amdgcn_ubfe(w1.x, 0u, p1)) - (s1 >> one);
                const uint32_t o2 = w2.y + __popc(__builtin_amdgcn_ubfe(w2.x, 0u, p2)) - (s2 >> one);
                const uint32_t z1 = oA[u] - o1, z2 = oB[u] - o2;
                const bool b1 = RA[u] & h, b2 = RB[u] & h;
                const bool u1 = b1 && z1 != 0;
                const bool u2 = b2 && min(nv - s2, h) > z2;  // zeros of the node past the prefix: suffix elements < R_B
                lA[u] = u1 ? l1 : lA[u];  // (the node start there is R & msk of that level: rebuilt from lA below)
                qA[u] = u1 ? z1 : qA[u];
                lB[u] = u2 ? l1 : lB[u];
                qB[u] = u2 ? z2 : qB[u];
                cA[u] += b1 ? 0u : o1;
                cB[u] += b2 ? 0u : o2;
                oA[u] = b1 ? o1 : z1;
                oB[u] = b2 ? o2 : z2;
            }
            h >>= 1;
            msk = (uint32_t)((int32_t)msk >> 1);
            l1 += 1;
            lvl += nw;
        }
    }
    // R's rank block: its node's first o entries are the prefix part's elements in it (mk: their ranks' bits), so
    // the ranks >= R among them finish the counts, and those below R hold the part's predecessor when any are there
    MT belA[NS], belB[NS];
    bool hitA[NS], hitB[NS], wrapA[NS], wrapB[NS];
    uint32_t l0 = WT_NONE;
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const uint32_t bA = RA[u] & ~BM, bB = RB[u] & ~BM, rA = RA[u] & BM, rB = RB[u] & BM;
        const MT mA = MK::load(mk, bA + (bA >> BB) + oA[u]), mB = MK::load(mk, bB + (bB >> BB) + oB[u]);
        cA[u] += MK::count_ge(mA, rA);
        cB[u] += MK::count_ge(mB, rB);
        W[u] += cA[u] + (n - RB[u]) - cB[u];
        belA[u] = MK::below(mA, rA);
        belB[u] = MK::below(MK::inv(mB), rB);
        // predecessors: in R's block when a part has an element below R there; else from the deepest branch-off
        // level down to a block (second descent: the prefix part takes the largest rank among the first qA entries of
        // node sA, the suffix part the largest among entries qB.. of node sB); a part with nothing below its bound
        // wraps, and its maximum is its largest rank overall: the same descent from the root (node 0, the part's
        // positions [0, d) or [d, n)). Levels no lane of the wave needs are skipped. (A per-d table of the parts'
        // largest ranks answered the wrap case with one read but cost 4 B per event of the row image.)
        hitA[u] = MK::any(belA[u]);
        hitB[u] = MK::any(belB[u]);
        wrapA[u] = d[u] > 0 && !hitA[u] && lA[u] == WT_NONE;
        wrapB[u] = d[u] < n && !hitB[u] && lB[u] == WT_NONE;
        if (wrapA[u]) {
            lA[u] = 0;
            qA[u] = d[u];
        }
        if (wrapB[u]) {
            lB[u] = 0;
            qB[u] = d[u];
        }
        const bool dA = d[u] > 0 && !hitA[u], dB = d[u] < n && !hitB[u];
        if (!dA) lA[u] = lb;
        if (!dB) lB[u] = lb;
        // the branch-off node: the left child recorded at level lA - 1 starts at R & ~(2^(K - lA + 1) - 1)
        sA[u] = RA[u] & ~((2u << (K - lA[u])) - 1u);
        sB[u] = RB[u] & ~((2u << (K - lB[u])) - 1u);
        l0 = min(l0, min(lA[u], lB[u]));
    }
#ifdef WT_ABL_PRED
    if (0)
#endif
    if (__builtin_amdgcn_ballot_w64(l0 < lb)) {
        for (uint32_t l = 0; l < lb; ++l) {
            if (!__builtin_amdgcn_ballot_w64(l >= l0)) continue;
            const uint32_t hs = 1u << (K - l - 1);
            const uint32_t h = wt_v(hs), h2 = wt_v(2 * hs), lv1 = wt_v(l);
            const uint2 *__restrict__ lvl = lv + l * nw;
#pragma unroll
            for (int u = 0; u < NS; ++u) {
                const uint32_t p1 = sA[u] + qA[u], p2 = sB[u] + qB[u];
                const uint2 w1 = lvl[p1 >> five], w2 = lvl[p2 >> five];
                const uint32_t o1 = w1.y + __popc(__builtin_amdgcn_ubfe(w1.x, 0u, p1)) - (sA[u] >> one);
                const uint32_t o2 = w2.y + __popc(__builtin_amdgcn_ubfe(w2.x, 0u, p2)) - (sB[u] >> one);
                const bool a1 = lv1 >= lA[u], a2 = lv1 >= lB[u];
                const bool g1 = a1 && o1 != 0;
                const bool g2 = a2 && min(nv - sB[u], h2) > h + o2;  // ones of the node past the prefix
                sA[u] += g1 ? h : 0u;
                qA[u] = g1 ? o1 : qA[u];
                sB[u] += g2 ? h : 0u;
                qB[u] = a2 ? (g2 ? o2 : qB[u] - o2) : qB[u];
            }
        }
    }
    // the descended lanes end in a block: the prefix part's elements are its first qA entries, the suffix part's the
    // entries from qB on (of the block's min(n - sB, 32))
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const MT vA = MK::load(mk, sA[u] + (sA[u] >> BB) + qA[u]);
        const MT vB = MK::low(MK::inv(MK::load(mk, sB[u] + (sB[u] >> BB) + qB[u])), min(nv - sB[u], BW));
        const uint32_t bA = RA[u] & ~BM, bB = RB[u] & ~BM;
        const uint32_t pA = hitA[u] ? bA + MK::top(belA[u]) : sA[u] + MK::top(vA);
        const uint32_t pB = hitB[u] ? bB + MK::top(belB[u]) : sB[u] + MK::top(vB);
        if (d[u] > 0) {
            const uint32_t t = Hm[u] + cm[pA] - (wrapA[u] ? m : 0u);
            const uint64_t k = ((uint64_t)t << 32) | (0xffffffffu - ev[pA]);
            key[u] = k > key[u] ? k : key[u];
        }
        if (d[u] < n) {
            const uint32_t t = Hm2[u] + cm[pB] - (wrapB[u] ? m : 0u);
            const uint64_t k = ((uint64_t)t << 32) | (0xffffffffu - ev[pB]);
            key[u] = k > key[u] ? k : key[u];
        }
        sum[u] += (uint64_t)d[u] * Hm[u] + (uint64_t)(n - d[u]) * Hm2[u];
    }
}

// ---------------------------------------------------------------------------------------------------------------
// top-k on the wavelet-tree path (k <= 64; order: sum desc as int64, seed asc; n_fault = 0 for this policy).
// Each workgroup's largest sum is the largest of a group of seeds, and the groups are disjoint, so the k-th largest
// of the group maxima (or of a subset of them) is a value at least k seeds reach: no seed below it is in the top k.
// One kernel (every block derives tau itself: cheaper than a launch) appends the seeds at or above tau (hundreds to
// a few thousand), and a one-block kernel sorts them (bitonic, LDS); more than WT_CAND candidates (heavy ties, e.g.
// maxInterval 1) take a slow exact selection there instead. The candidate
// counter resets itself. (A "last block" handing tau or the ranking to the final workgroup of a kernel needs
// device-scope fences, i.e. L2 writebacks on every XCD: +40 us on the sweep.)
// ---------------------------------------------------------------------------------------------------------------
constexpr uint32_t WT_CAND = 4096;
constexpr uint32_t WT_MAX_GROUPS = 256 * 8;
struct WtTopkState {
    uint32_t n_cand, pad[3];
    unsigned long long gmax[WT_MAX_GROUPS];
    unsigned long long cand_key[WT_CAND];
    unsigned long long cand_idx[WT_CAND];
};

#ifdef WT_TRACE
// timing-only builds (-DWT_TRACE, G = 1): wall_clock64 per (row, wave) at the kernel start [9], after staging [0] and
// at the end of each of up to 8 chunks [1..8]; read with nmz_debug_wt_trace (tools/k1_trace.py --wt)
__device__ unsigned long long g_wt_trace[256][16][10];
#define WT_TSTAMP(slot)                                                                                      \
    do {                                                                                                     \
        if ((threadIdx.x & 63) == 0 && blockIdx.x < 256 && (slot) < 10)                                      \
            g_wt_trace[blockIdx.x][threadIdx.x >> 6][(slot)] = wall_clock64();                               \
    } while (0)
#else
#define WT_TSTAMP(slot) \
    do {                \
    } while (0)
#endif

#ifndef WT_PRIO_TAIL
#define WT_PRIO_TAIL 0  // 8, 16, 32: no change in K1 (profiles/r05/k1/prio_ab)
#endif

// G workgroups per row L: each stages the row image into LDS and takes a contiguous share of the row's chunks of
// 64 NS seeds (NS per lane), which its waves take one at a time from an LDS counter.
// The row image (~84 KB at configs[1]) allows one workgroup (16 waves, 4 per SIMD) per CU, so registers beyond the 64
// that 8 waves/SIMD would need cost no occupancy; NMZ_WT_WAVES=4 lets the compiler schedule with up to 128 (A/B)
#ifndef NMZ_WT_WAVES
#define NMZ_WT_WAVES 0
#endif
#if NMZ_WT_WAVES > 0
#define NMZ_WT_ATTR __attribute__((amdgpu_waves_per_eu(NMZ_WT_WAVES, NMZ_WT_WAVES)))
#else
#define NMZ_WT_ATTR
#endif
template <bool BIG, int NS, int BB>
__global__ __launch_bounds__(1024) NMZ_WT_ATTR void k_replayable_sweep_wt(
    const uint32_t *__restrict__ bucket_off, const uint64_t *__restrict__ sorted_h0,
    const uint32_t *__restrict__ sorted_idx, const uint4 *__restrict__ table, uint32_t E,
    const uint4 *__restrict__ blob, uint32_t rb16, const unsigned long long *__restrict__ rowsum,
    const WtClass *__restrict__ classes, uint32_t n_classes, uint32_t m, uint64_t mu, uint32_t m_k64, uint32_t msh,
    uint32_t G, nmz_sched_stats *__restrict__ stats, unsigned long long *__restrict__ span,
    uint64_t *__restrict__ sums, WtTopkState *__restrict__ tk, uint32_t k) {
    constexpr uint32_t CS = 64 * NS;  // seeds per chunk
    extern __shared__ uint4 wt_lds[];
    const uint32_t L = blockIdx.x / G, g = blockIdx.x % G;
    const uint32_t s0 = bucket_off[L], s1 = bucket_off[L + 1];
    const uint32_t nch = (s1 - s0 + CS - 1) / CS;
    const uint32_t c0 = g * nch / G, c1 = (g + 1) * nch / G;
    uint32_t *ctr = reinterpret_cast<uint32_t *>(wt_lds + rb16);
    if (tk && blockIdx.x == 0 && threadIdx.x == 0) tk->n_cand = 0;  // the top-k scan after this sweep appends
    if (c0 == c1) {  // no seeds (an empty group: the smallest key)
        if (tk && threadIdx.x == 0) tk->gmax[blockIdx.x] = 0ull;
        return;
    }
    if (span && threadIdx.x == 0) atomicMax(span, ~(unsigned long long)wall_clock64());
    WT_TSTAMP(9);
    {
        const uint4 *__restrict__ src = blob + (uint64_t)L * rb16;
        // every load of a pass in flight at once (indices clamped to the image, stores unconditional)
        constexpr uint32_t B = 8;
        const uint32_t nt = blockDim.x;
        for (uint32_t i0 = 0; i0 < rb16; i0 += B * nt) {
            uint4 v[B];
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) v[k] = src[min(i0 + k * nt + threadIdx.x, rb16 - 1)];
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) wt_lds[min(i0 + k * nt + threadIdx.x, rb16 - 1)] = v[k];
        }
        if (threadIdx.x == 0) {
            *ctr = c0;
            ctr[2] = ctr[3] = 0;  // the workgroup's largest sum key
        }
    }
    __syncthreads();
    WT_TSTAMP(0);
#ifdef WT_TRACE
    uint32_t n_done = 0;
#endif
    const char *img = reinterpret_cast<const char *>(wt_lds);
    const uint4 *__restrict__ row = table + (uint64_t)L * E;
    const uint64_t rsum = rowsum[L];
    const uint32_t lane = threadIdx.x & 63;
    WtVConst vc;
#pragma unroll
    for (int r = 0; r < 5; ++r) vc.st4[r] = wt_v(4u << r);
    // chunks from the LDS counter; the next chunk's seeds and indices are loaded while this one runs
    uint32_t ch = 0;
    if (lane == 0) ch = atomicAdd(ctr, 1u);
    ch = __builtin_amdgcn_readfirstlane(ch);
    uint64_t h0n[NS];
    uint32_t idxn[NS];
#pragma unroll
    for (int u = 0; u < NS; ++u) {
        const uint32_t jn = min(s0 + ch * CS + u * 64 + lane, s1 - 1);  // past the share: a valid seed, unused
        h0n[u] = sorted_h0[jn];
        idxn[u] = sorted_idx[jn];
    }
    while (ch < c1) {
#if WT_PRIO_TAIL > 0
        // the row's last chunks: the SIMD arbiter serves older waves first, so a chunk taken late by a young wave
        // waits behind them and then runs alone at the end of the row; raising the priority of the waves on the
        // last chunks lets them finish together with the rest
        if (ch + WT_PRIO_TAIL >= c1) __builtin_amdgcn_s_setprio(3);
#endif
        const uint32_t j0 = s0 + ch * CS + lane;
        uint64_t h0[NS];
        uint32_t idx[NS];
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            h0[u] = h0n[u];
            idx[u] = idxn[u];
        }
        uint32_t chn = 0;
        if (lane == 0) chn = atomicAdd(ctr, 1u);
        chn = __builtin_amdgcn_readfirstlane(chn);
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const uint32_t jn = min(s0 + chn * CS + u * 64 + lane, s1 - 1);
            h0n[u] = sorted_h0[jn];
            idxn[u] = sorted_idx[jn];
        }
        uint64_t sum[NS], key[NS];
        uint32_t W[NS];
#pragma unroll
        for (int u = 0; u < NS; ++u) sum[u] = key[u] = W[u] = 0;
        for (uint32_t c = 0; c < n_classes; ++c)
            wt_seed_class<BIG, NS, BB>(vc, classes[c], img, row, h0, m, mu, m_k64, msh, sum, W, key);
        uint64_t km = 0;  // the chunk's largest sum, in the top-k's order (int64, as an order-preserving u64 key)
#pragma unroll
        for (int u = 0; u < NS; ++u) {
            const uint32_t j = j0 + u * 64;
            const uint64_t total = sum[u] + rsum - (uint64_t)W[u] * m;
            if (j < s1) {
                const uint64_t kk = total ^ (1ull << 63);
                km = kk > km ? kk : km;
                if (sums) sums[j] = total;  // in sorted order: the wave's 64 writes coalesce (by seed index they
                                            // scatter, one 64-B line per seed: +20 us on the step)
                nmz_sched_stats st;
                st.sum_delay_ns = total;
                st.max_delay_ns = (int64_t)(key[u] >> 32);
                st.argmax_event = ~(uint32_t)key[u];
                st.n_fault = 0;
                st.first_fault = NMZ_NONE;
                st.flags = 0;
                stats[idx[u]] = st;
            }
        }
        if (tk) {
            for (int o = 32; o; o >>= 1) {
                const uint64_t v = __shfl_xor(km, o, 64);
                km = v > km ? v : km;
            }
            if (lane == 0) atomicMax(reinterpret_cast<unsigned long long *>(ctr + 2), (unsigned long long)km);
        }
#ifdef WT_TRACE
        if (++n_done <= 8) WT_TSTAMP(n_done);
#endif
        ch = chn;
    }
    if (span || tk) {
        __syncthreads();
        if (span && threadIdx.x == 0) atomicMax(span + 1, (unsigned long long)wall_clock64());
        if (tk && threadIdx.x == 0) tk->gmax[blockIdx.x] = *reinterpret_cast<const unsigned long long *>(ctr + 2);
    }
}

__device__ __forceinline__ bool wt_better(unsigned long long ka, uint64_t sa, unsigned long long kb, uint64_t sb) {
    return ka > kb || (ka == kb && sa < sb);
}

// every block: tau = the k-th largest key of min(n, 512) groups sampled evenly over all rows (a subset's k-th largest
// is at most the whole set's, so tau stays a value at least k seeds reach; ~k n / 512 of the groups' maxima lie
// above it), by counting; then a grid-stride scan of the sweep's sums appending the seeds at or above tau (hundreds
// to a few thousand: a row whose sums peak high holds many seeds near its peak). (The first 256 groups alone -- a few rows -- let one configs[1] trace in 17 overflow the
// candidate list into the slow exact selection: 50 ms.)
__global__ __launch_bounds__(256) void k_wt_topk_scan(const uint64_t *__restrict__ sums,
                                                      const uint32_t *__restrict__ sorted_idx, uint64_t S, uint32_t n,
                                                      uint32_t k, WtTopkState *__restrict__ tk) {
    constexpr uint32_t PF = 16;  // sums per thread loaded before they are needed (their latency overlaps tau)
    constexpr uint32_t NS = 512;  // sampled groups
    __shared__ unsigned long long g[NS];
    __shared__ unsigned long long tau_s;
    const uint32_t m = min(n, NS);
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    uint64_t v[PF];
#pragma unroll
    for (uint32_t r = 0; r < PF; ++r) {
        const uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x + r * stride;
        v[r] = i < S ? sums[i] : 0ull;
    }
    for (uint32_t i = threadIdx.x; i < m; i += 256) g[i] = tk->gmax[(uint64_t)i * n / m];
    // fewer groups than k: every seed is a candidate (tau 0); else the k-th largest sampled maximum = the smallest
    // of those with fewer than k others above them (one count per value, no tie count)
    if (threadIdx.x == 0) tau_s = m >= k ? ~0ull : 0ull;
    __syncthreads();
    if (m >= k) {
        unsigned long long best = ~0ull;
        for (uint32_t i = threadIdx.x; i < m; i += 256) {
            const unsigned long long x = g[i];
            uint32_t gt = 0;
#pragma unroll 8
            for (uint32_t j = 0; j < m; ++j) gt += g[j] > x;
            if (gt < k) best = x < best ? x : best;
        }
        if (best != ~0ull) atomicMin(&tau_s, best);
    }
    __syncthreads();
    const unsigned long long t = tau_s;
    const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    // the block's candidates of one round of PF sums per thread are counted in registers and block-scanned, and ONE
    // returning atomic per block reserves their range: a returning atomic per candidate wave (the previous form,
    // hundreds to thousands on one word at ~11 ns each) serialised the scan
    __shared__ uint32_t wsum[4], base_s;
    for (uint64_t i0 = (uint64_t)blockIdx.x * 256; i0 < S; i0 += PF * stride) {
        uint32_t flags = 0;
#pragma unroll
        for (uint32_t r = 0; r < PF; ++r) {
            const uint64_t i = i0 + threadIdx.x + r * stride;
            if (i0 != (uint64_t)blockIdx.x * 256) v[r] = i < S ? sums[i] : 0ull;  // past the first PF rounds
            const unsigned long long key = v[r] ^ (1ull << 63);
            flags |= (i < S && key >= t) ? 1u << r : 0u;
        }
        const uint32_t n = __popc(flags);
        uint32_t a = n;
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t x = __shfl_up(a, d, 64);
            if (lane >= d) a += x;
        }
        if (lane == 63) wsum[w] = a;
        __syncthreads();
        uint32_t pre = 0, total = 0;
        for (uint32_t x = 0; x < 4; ++x) {
            pre += x < w ? wsum[x] : 0u;
            total += wsum[x];
        }
        if (total) {
            if (threadIdx.x == 0) base_s = atomicAdd(&tk->n_cand, total);
            __syncthreads();
            uint32_t pos = base_s + pre + a - n;
#pragma unroll
            for (uint32_t r = 0; r < PF; ++r) {
                if (flags >> r & 1u) {
                    if (pos < WT_CAND) {
                        const uint64_t i = i0 + threadIdx.x + r * stride;
                        tk->cand_key[pos] = v[r] ^ (1ull << 63);
                        tk->cand_idx[pos] = sorted_idx[i];
                    }
                    ++pos;
                }
            }
        }
        __syncthreads();  // wsum and base_s are rewritten by the next round
    }
}

// one block: sort the candidates and write the top k (past WT_CAND candidates -- heavy ties, e.g. maxInterval 1 --
// select them one rank at a time over every seed: exact, slow); resets the candidate counter
#ifndef NMZ_WT_SEL_THREADS
#define NMZ_WT_SEL_THREADS 512
#endif
constexpr uint32_t WT_SEL_THREADS = NMZ_WT_SEL_THREADS;
constexpr uint32_t WT_SEL_CHUNK = 2048, WT_SEL_KEEP = (WT_CAND / WT_SEL_CHUNK) * 64;
__global__ __launch_bounds__(WT_SEL_THREADS) void k_wt_topk_select(const uint64_t *__restrict__ sums,
                                                                   const uint32_t *__restrict__ sorted_idx, uint64_t S,
                                                                   uint64_t seed0, uint32_t k,
                                                                   WtTopkState *__restrict__ tk,
                                                                   nmz_topk_entry *__restrict__ out) {
    constexpr uint32_t NT = WT_SEL_THREADS, NW = NT / 64;
    // candidates sorted in chunks of WT_SEL_CHUNK, each chunk's best k kept aside, then the kept ones sorted: 26 KB of
    // LDS instead of 48 for one sort of WT_CAND, so the kernel fits beside a K1 workgroup whose row image has wider
    // rank blocks (it waits for a whole CU otherwise: +8 us per configs[1] step)
    __shared__ unsigned long long ck[WT_SEL_CHUNK];
    __shared__ uint32_t ci[WT_SEL_CHUNK];
    __shared__ unsigned long long sk[WT_SEL_KEEP];
    __shared__ uint32_t si[WT_SEL_KEEP];
    __shared__ unsigned long long bk[NW], bs[NW];
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t c = tk->n_cand;
    auto sentinel = [] {
        nmz_topk_entry e;
        e.seed = UINT64_MAX;
        e.sum_delay_ns = INT64_MIN;
        e.n_fault = 0;
        e.first_fault = NMZ_NONE;
        return e;
    };
    if (c <= WT_CAND) {
        // every seed at or above the scan's tau is a candidate (hundreds to a few thousand: a row whose sums peak
        // high holds many near its peak): a bitonic sort of (key desc, seed asc) in LDS, padded with key 0 (a real
        // key has its top bit set: sums are non-negative)
        // bitonic sort of ck/ci[0, p2) (key desc, seed asc; padding last)
        auto sort = [&](uint32_t p2) {
            for (uint32_t kk = 2; kk <= p2; kk <<= 1)
                for (uint32_t j = kk >> 1; j; j >>= 1) {
                    __syncthreads();
                    for (uint32_t i = threadIdx.x; i < p2; i += NT) {
                        const uint32_t l = i ^ j;
                        if (l > i) {
                            const unsigned long long a = ck[i], b = ck[l];
                            const uint32_t ia = ci[i], ib = ci[l];
                            // l better than i
                            const bool lb = b > a || (b == a && b != 0 && seed0 + ib < seed0 + ia);
                            if (lb == ((i & kk) == 0)) {
                                ck[i] = b;
                                ck[l] = a;
                                ci[i] = ib;
                                ci[l] = ia;
                            }
                        }
                    }
                }
            __syncthreads();
        };
        auto pow2 = [](uint32_t x) {
            uint32_t p = 1;
            while (p < x) p <<= 1;
            return p;
        };
        const uint32_t nch = c > WT_SEL_CHUNK ? (c + WT_SEL_CHUNK - 1) / WT_SEL_CHUNK : 1;
        for (uint32_t q = 0; q < nch; ++q) {
            const uint32_t lo = q * WT_SEL_CHUNK, cc = min(c - lo, WT_SEL_CHUNK), p2 = pow2(cc);
            for (uint32_t i = threadIdx.x; i < p2; i += NT) {
                ck[i] = i < cc ? tk->cand_key[lo + i] : 0ull;
                ci[i] = i < cc ? (uint32_t)tk->cand_idx[lo + i] : ~0u;
            }
            sort(p2);
            if (nch > 1) {  // the chunk's best k aside (a seed outside them is beaten by k of this chunk alone)
                for (uint32_t i = threadIdx.x; i < k; i += NT) {
                    sk[q * k + i] = ck[i];
                    si[q * k + i] = ci[i];
                }
                __syncthreads();
            }
        }
        if (nch > 1) {
            const uint32_t p2 = pow2(nch * k);
            for (uint32_t i = threadIdx.x; i < p2; i += NT) {
                ck[i] = i < nch * k ? sk[i] : 0ull;
                ci[i] = i < nch * k ? si[i] : ~0u;
            }
            sort(p2);
        }
        for (uint32_t r = threadIdx.x; r < k; r += NT) {
            if (r < c) {
                nmz_topk_entry e;
                e.seed = seed0 + ci[r];  // seeds wrap as elsewhere
                e.sum_delay_ns = (int64_t)(ck[r] ^ (1ull << 63));
                e.n_fault = 0;
                e.first_fault = NMZ_NONE;
                out[r] = e;
            } else {
                out[r] = sentinel();  // fewer seeds than k
            }
        }
    } else {
        // exact selection one rank at a time: the best entry after the previous one in (key desc, seed asc)
        unsigned long long pk = ~0ull, ps = 0;
        bool first_rank = true;
        for (uint32_t r = 0; r < k; ++r) {
            unsigned long long mk = 0, ms = ~0ull;
            bool any = false;
            for (uint64_t i = threadIdx.x; i < S; i += NT) {
                const unsigned long long key = sums[i] ^ (1ull << 63), sd = seed0 + sorted_idx[i];
                const bool after = first_rank || wt_better(pk, ps, key, sd);
                if (after && (!any || wt_better(key, sd, mk, ms))) {
                    mk = key;
                    ms = sd;
                    any = true;
                }
            }
            if (!any) mk = 0, ms = ~0ull;
            for (int o = 32; o; o >>= 1) {
                const unsigned long long ok = __shfl_xor(mk, o, 64), os = __shfl_xor(ms, o, 64);
                const bool oany = __shfl_xor((int)any, o, 64);
                if (oany && (!any || wt_better(ok, os, mk, ms))) {
                    mk = ok;
                    ms = os;
                    any = true;
                }
            }
            __syncthreads();
            if (lane == 0) {
                bk[threadIdx.x >> 6] = any ? mk : 0;
                bs[threadIdx.x >> 6] = any ? ms : ~0ull;
                if (!any) bs[threadIdx.x >> 6] = ~0ull, bk[threadIdx.x >> 6] = 0;
            }
            __syncthreads();
            // the block's best (empty slots hold key 0, seed ~0: never better than a real entry of key 0 with a
            // smaller seed; a real entry of key 0 and seed ~0 is found by the any flags below)
            unsigned long long bestk = 0, bests = ~0ull;
            bool found = false;
            for (uint32_t w = 0; w < NW; ++w) {
                const bool real = !(bk[w] == 0 && bs[w] == ~0ull);
                if (real && (!found || wt_better(bk[w], bs[w], bestk, bests))) {
                    bestk = bk[w];
                    bests = bs[w];
                    found = true;
                }
            }
            if (!found) {
                for (uint32_t q = r + threadIdx.x; q < k; q += NT) out[q] = sentinel();
                break;
            }
            if (threadIdx.x == 0) {
                nmz_topk_entry e;
                e.seed = bests;
                e.sum_delay_ns = (int64_t)(bestk ^ (1ull << 63));
                e.n_fault = 0;
                e.first_fault = NMZ_NONE;
                out[r] = e;
            }
            pk = bestk;
            ps = bests;
            first_rank = false;
        }
    }
    __syncthreads();
    if (threadIdx.x == 0) tk->n_cand = 0;
}

// ---------------------------------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------------------------------
static uint32_t bitlen(uint64_t x) {
    uint32_t b = 0;
    while (x) {
        ++b;
        x >>= 1;
    }
    return b;
}

// read at every plan build (tests switch it per plan)
bool wt_enabled() {
    const char *e = ab_env("NMZ_REPLAY_WT");
    return !(e && std::string(e) == "0");
}

// workgroups per row and threads per workgroup (A/B knobs NMZ_WT_G = 1|2|4|8, NMZ_WT_THREADS = 64..1024)
static uint32_t wt_groups() {
    static const uint32_t g = [] {
        // one workgroup per row leaves half of each CU's wave slots and LDS to the step's other kernels (the seed
        // prefix, bucketing and top-k of the neighbouring pipelined steps): configs[1] step 0.116 -> 0.113 ms with
        // the fused top-k (profiles/r03y_wt_groups_ab.json); alone, 2 per row are 2 % faster
        const char *e = ab_env("NMZ_WT_G");
        const int v = e ? atoi(e) : 1;
        return (uint32_t)((v == 1 || v == 2 || v == 4 || v == 8) ? v : 1);
    }();
    return g;
}
static uint32_t wt_threads() {
    static const uint32_t t = [] {
        const char *e = ab_env("NMZ_WT_THREADS");
        const int v = e ? atoi(e) : 1024;
        return (uint32_t)((v >= 64 && v <= 1024 && v % 64 == 0) ? v : 1024);
    }();
    return t;
}

// the widest rank blocks a plan may take: 64 ranks (NMZ_WT_BB = 5 | 6 | 7, A/B and tests; read at every plan build)
static uint32_t wt_max_bb() {
    const char *e = ab_env("NMZ_WT_BB");
    const int v = e ? atoi(e) : 6;
    return (uint32_t)((v >= 5 && v <= 7) ? v : 6);
}

constexpr size_t WT_BUILD_LDS = WT_NMAX * 8 * 2 + WT_NMAX / 2 * 4 + 2 * (WT_NMAX / 32 + 4) * 4 + 520 * 4 +
                                WT_BW * 8 + 16;

bool wt_layout(WtState &w, nmz_ctx *ctx, uint32_t E, const ClassInfo *cls, uint32_t n_cls, const ModParams &mod,
               bool fused, std::vector<WtClass> &oc) {
    w.on = false;
    if (!wt_enabled() || !mod.m32ok || E == 0 || E > 65536) return false;
    if (fused) {  // every class is one segment the plan kernel sorts itself
        for (uint32_t c = 0; c < n_cls; ++c)
            if (cls[c].count > WT_NMAX - 1) return false;
    }
    auto r16 = [](uint64_t b) { return (b + 15) & ~15ull; };
    // segments: a class of 4,096 events or more (the plan kernel sorts < 4,096 keys in LDS) splits into near-equal
    // C-sorted sub-segments, each one a segment in its own right (every decision of it is (base + Cm) mod m with
    // the same carry rule C > ~H, just over fewer events)
    std::vector<ClassInfo> seg;
    for (uint32_t c = 0; c < n_cls; ++c) {
        const uint32_t n = cls[c].count, parts = (n + WT_NMAX - 2) / (WT_NMAX - 1);
        for (uint32_t k = 0, lo = 0; k < parts; ++k) {
            const uint32_t len = n / parts + (k < n % parts ? 1u : 0u);
            seg.push_back(ClassInfo{cls[c].pn, cls[c].start + lo, len});
            lo += len;
        }
    }
    n_cls = (uint32_t)seg.size();
    auto layout = [&](uint32_t bb) -> uint64_t {
    oc.assign(n_cls, WtClass{});
    uint64_t off = 0;
    for (uint32_t c = 0; c < n_cls; ++c) {
        WtClass &o = oc[c];
        o.pn = seg[c].pn;
        o.start = seg[c].start;
        o.n = seg[c].count;
        if (o.n <= WT_BRUTE) continue;
        o.K = bitlen(o.n);  // 2^K > n >= every bound R
        o.nw = o.n / 32 + 1;
        o.o_lv = (uint32_t)off;
        off += r16((uint64_t)wt_levels(o.K, bb) * o.nw * 8);
        o.o_cm = (uint32_t)off;
        off += r16((uint64_t)(o.n + WT_PAD) * 4);
        o.o_chi = (uint32_t)off;
        off += r16((uint64_t)(o.n + WT_PAD) * 4);
        o.o_e = (uint32_t)off;
        off += r16((uint64_t)o.n * 2);
        o.o_im = (uint32_t)off;
        off += r16(257 * 2);
        o.o_ic = (uint32_t)off;
        off += r16(256 * 2);
        o.o_mk = (uint32_t)off;
        off += r16(wt_mask_bytes(o.n, bb));
    }
    return off;
    };
    // the widest rank blocks whose row image fits LDS (NMZ_WT_BB caps the width, A/B and tests)
    uint32_t bb = wt_max_bb();
    uint64_t off = layout(bb);
    while (bb > 5 && std::max<uint64_t>(16, r16(off)) + 16 > WT_LDS_MAX) off = layout(--bb);
    {  // the plan kernel's dispatch order: segments by size, largest first
        std::vector<uint32_t> ord(n_cls);
        std::iota(ord.begin(), ord.end(), 0u);
        std::stable_sort(ord.begin(), ord.end(), [&](uint32_t a, uint32_t b) { return oc[a].n > oc[b].n; });
        for (uint32_t r = 0; r < n_cls; ++r) oc[r].order = ord[r];
    }
    const uint64_t rb = std::max<uint64_t>(16, r16(off));
    if (rb + 16 > WT_LDS_MAX) return false;
    // function attributes are per device: once per context (a context owns one device; its calls are serialised)
    if (!ctx->wt_lds_attr) {
        for (const void *f : {reinterpret_cast<const void *>(k_replayable_sweep_wt<false, 1, 5>),
                              reinterpret_cast<const void *>(k_replayable_sweep_wt<true, 1, 5>),
                              reinterpret_cast<const void *>(k_replayable_sweep_wt<false, 1, 6>),
                              reinterpret_cast<const void *>(k_replayable_sweep_wt<true, 1, 6>),
                              reinterpret_cast<const void *>(k_replayable_sweep_wt<false, 1, 7>),
                              reinterpret_cast<const void *>(k_replayable_sweep_wt<true, 1, 7>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<false, 5>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<true, 5>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<false, 6>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<true, 6>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<false, 7>),
                              reinterpret_cast<const void *>(k_replayable_wt_build<true, 7>)})
            if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WT_LDS_MAX) != hipSuccess) {
                (void)hipGetLastError();  // not sticky for the launches that follow: keep the order-query sweep
                return false;
            }
        ctx->wt_lds_attr = true;
    }
    w.rb16 = (uint32_t)(rb / 16);
    w.bb = bb;
    w.n_classes = n_cls;
    w.msh = mod.m32 > 255 ? bitlen(mod.m32) - 8 : 0;
    return true;
}

int wt_launch(WtState &w, const uint4 *d_table, uint32_t E, const ModParams &mod, hipStream_t st,
              const WtPlanHints *hints, WtClass *d_cls, unsigned long long *d_rowsum, bool sync) {
    NMZ_TRY(w.mem.ensure(Carve::bytes_for(256 * (size_t)w.rb16, 16)));
    w.d_blob = w.mem.as<uint4>();
    w.d_rowsum = d_rowsum;
    w.d_classes = d_cls;
    WtHints hz{};
    if (hints)
        hz = WtHints{hints->hoff, hints->hbytes, hints->perm, mod.m, mod.mu, hints->table, hints->zero0, hints->n_zero0,
                     hints->zero1, hints->n_zero1};
    auto kern = hints ? (w.bb == 7 ? k_replayable_wt_build<true, 7>
                         : w.bb == 6 ? k_replayable_wt_build<true, 6> : k_replayable_wt_build<true, 5>)
                      : (w.bb == 7 ? k_replayable_wt_build<false, 7>
                         : w.bb == 6 ? k_replayable_wt_build<false, 6> : k_replayable_wt_build<false, 5>);
    hipLaunchKernelGGL(kern, dim3(w.n_classes, 256), dim3(WT_BT), WT_BUILD_LDS, st, hints ? nullptr : d_table, E,
                       d_cls, w.msh, bitlen(mod.m32), w.d_blob, w.rb16, d_rowsum, hz);
    NMZ_HIP(hipGetLastError());
    if (sync) NMZ_HIP(hipStreamSynchronize(st));  // the plan is complete when it is returned
    w.on = true;
    return NMZ_OK;
}

int wt_build(WtState &w, nmz_ctx *ctx, const uint4 *d_table, uint32_t E, const ClassInfo *cls, uint32_t n_cls,
             const ModParams &mod, hipStream_t st) {
    std::vector<WtClass> oc;
    if (!wt_layout(w, ctx, E, cls, n_cls, mod, false, oc)) return NMZ_OK;
    // classes and row sums in their own buffer (the fused path uploads them with the plan's inputs)
    NMZ_TRY(w.aux.ensure(Carve::bytes_for(256, 8) + Carve::bytes_for(oc.size(), sizeof(WtClass))));
    Carve cv(w.aux.ptr);
    unsigned long long *d_rowsum = cv.take<unsigned long long>(256);
    WtClass *d_cls = cv.take<WtClass>(oc.size());
    NMZ_HIP(hipMemsetAsync(d_rowsum, 0, 256 * 8, st));
    NMZ_TRY(ctx->pin[1].ensure(oc.size() * sizeof(WtClass)));
    std::memcpy(ctx->pin[1].ptr, oc.data(), oc.size() * sizeof(WtClass));
    NMZ_HIP(hipMemcpyAsync(d_cls, ctx->pin[1].ptr, oc.size() * sizeof(WtClass), hipMemcpyHostToDevice, st));
    NMZ_TRY(ctx->pin[1].mark(st));
    return wt_launch(w, d_table, E, mod, st, nullptr, d_cls, d_rowsum, true);
}

size_t wt_topk_scratch_bytes(uint64_t S) {
    return Carve::bytes_for(1, sizeof(WtTopkState)) + Carve::bytes_for(S, 8);
}

// the selection after a sweep that ran with this scratch (its per-seed sums and per-workgroup largest sums)
int wt_topk(hipStream_t st, void *scratch, const uint32_t *sorted_idx, uint64_t S, uint64_t seed0, uint32_t k,
            nmz_topk_entry *d_out) {
    NMZ_CHECK(k >= 1 && k <= 64, "internal: wt_topk takes 1 <= k <= 64");
    Carve cv(scratch);
    WtTopkState *tk = cv.take<WtTopkState>(1);
    const uint64_t *sums = cv.take<uint64_t>(S);
    // (64 blocks, for less of the per-block tau derivation, made the configs[1] step slower: 0.072 -> 0.077 ms, the
    // longer scan delaying its stream's next step)
    const unsigned blocks = (unsigned)std::min<uint64_t>(ceil_div(S, 256), 256);
    hipLaunchKernelGGL(k_wt_topk_scan, dim3(blocks), dim3(256), 0, st, sums, sorted_idx, S, 256 * wt_groups(), k, tk);
    hipLaunchKernelGGL(k_wt_topk_select, dim3(1), dim3(WT_SEL_THREADS), 0, st, sums, sorted_idx, S, seed0, k, tk,
                       d_out);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// topk_scratch (wt_topk_scratch_bytes(S)) or nullptr: the sweep also leaves per-seed sums and per-workgroup largest
// sums there for wt_topk
int wt_sweep(const WtState &w, nmz_ctx *ctx, hipStream_t st, const Buckets &b, const uint4 *d_table, uint32_t E,
             const ModParams &mod, nmz_sched_stats *d_stats, uint64_t S, void *topk_scratch, uint32_t k) {
    WtTopkState *tk = nullptr;
    uint64_t *sums = nullptr;
    if (topk_scratch) {
        Carve cv(topk_scratch);
        tk = cv.take<WtTopkState>(1);
        sums = cv.take<uint64_t>(S);
    }
    const uint32_t G = wt_groups(), nt = wt_threads();
    KernelTimer kt(ctx, st, "replayable_sweep");
    unsigned long long *span = kt.span();
    const bool big = mod.m32 >= 0x80000000u;
    // one seed per lane: two (NS = 2, 106 VGPRs) measured slower, K1 span 0.074 vs 0.059 ms
    // (profiles/r04/k1_ns2_rejected/)
    auto kern = big ? (w.bb == 7 ? k_replayable_sweep_wt<true, 1, 7>
                       : w.bb == 6 ? k_replayable_sweep_wt<true, 1, 6> : k_replayable_sweep_wt<true, 1, 5>)
                    : (w.bb == 7 ? k_replayable_sweep_wt<false, 1, 7>
                       : w.bb == 6 ? k_replayable_sweep_wt<false, 1, 6> : k_replayable_sweep_wt<false, 1, 5>);
    const size_t lds = w.rb16 * 16u + 16u;
    hipLaunchKernelGGL(kern, dim3(256 * G), dim3(nt), lds, st, b.offset, b.sorted_h0, b.sorted_idx,
                       d_table, E, w.d_blob, w.rb16, w.d_rowsum, static_cast<const WtClass *>(w.d_classes),
                       w.n_classes, mod.m32, mod.mu, mod.m_k64, w.msh, G, d_stats, span, sums, tk, k);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz

#ifdef WT_TRACE
extern "C" int nmz_debug_wt_trace(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nmz::g_wt_trace), sizeof(nmz::g_wt_trace)) == hipSuccess ? 0 : -1;
}
#endif

#ifdef WT_BUILD_TRACE
extern "C" int nmz_debug_wt_build_trace(unsigned long long *out, uint32_t n) {
    const uint32_t m = std::min<uint32_t>(n, nmz::WT_TRACE_WGS * nmz::WT_TRACE_PHASES);
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nmz::g_wt_build_trace), m * 8) == hipSuccess ? 0 : -1;
}
#endif
