// K4 -- wide-band bit-parallel banded Levenshtein (configs[4]: 64k-event
// traces, w = 4096): one trace pair per wave, the band spread over the lanes.
//
// Same recurrence and boundary argument as ed_bv.hip (diagonal band,
// virtual rows, +1 deltas at the band edges, T = value of the band's top
// cell, cut-off on T - popcount(M)).  Here the band's 2w bits (w = 1024*KL)
// are split over the 64 lanes, KL words per lane: bit 32*(KL*l + k) + b of
// the band lives in lane l, word k.  Per column the wave does
//   * one coalesced 4(KL+1)-byte-per-lane load of the query's match bitmap
//     row for the candidate symbol b_j (uniform across the wave), from a
//     per-trace table in HBM that stays L2-resident (pairs sharing a query
//     trace run back to back on one XCD), prefetched 8 columns ahead;
//   * the (Eq & P) + P addition with a cross-lane carry: each lane's carry
//     out (generate) and all-ones sum (propagate) are ballots, and the carry
//     into every lane is one 64-bit scalar add: C = (G + (G|Pr)) ^ G ^ (G|Pr);
//   * the one-bit band slide Xs = Xv >> 1, whose top bit comes from the next
//     lane through a DPP wave_shl:1 move.
// ~55 VALU instructions per column cover 2w+1 = 8193 DP cells.
// Bands 64 < w <= 8192 run on the kernel of the smallest W = 1024 * 2^k >= w with w applied at run time
// (length band, cut-off, clamp; exact as in ed_bv.hip: min(D_W, w + 1) = min(D_w, w + 1)).
#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

typedef uint32_t u32x4u __attribute__((ext_vector_type(4), aligned(4)));

__device__ __forceinline__ uint32_t wa_alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

__device__ __forceinline__ uint32_t wave_sum_u32(uint32_t v) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) v += (uint32_t)__shfl_xor((int)v, off, 64);
    return __builtin_amdgcn_readfirstlane(v);  // uniform: keeps dependent control flow scalar
}

__device__ __forceinline__ void wide_knn_insert(uint64_t *list, uint32_t k, uint64_t key) {
    if (key >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    for (uint32_t s = 0; s < k; ++s) {
        const uint64_t old = atomicMin((unsigned long long *)&list[s], (unsigned long long)key);
        if (old == UINT64_MAX) return;
        key = old > key ? old : key;
    }
}

template <int KL>
struct WideState {
    uint32_t P[KL], M[KL];
    uint32_t acc;  // lane 0: bit per column (M | Xh) & 1 = 1 - increment of T
};

// one column; d = this lane's KL+1 dwords of Eq, already loaded
template <int KL>
__device__ __forceinline__ void wide_column(WideState<KL> &S, const uint32_t (&d)[KL + 1], uint32_t t,
                                            uint32_t lane) {
    uint32_t Eq[KL], Xv[KL], X[KL], Xh[KL], Ph[KL], Mh[KL], Xs[KL];
#pragma unroll
    for (int k = 0; k < KL; ++k) Eq[k] = wa_alignbit(d[k + 1], d[k], t);
#pragma unroll
    for (int k = 0; k < KL; ++k) Xv[k] = Eq[k] | S.M[k];
    // X = (Eq & P) + P over the whole band: per-lane carry chain (carry out of
    // every lane = the generate mask G), then the carry into each lane from one
    // 64-bit scalar add over the lane masks, fed back as the chains' carry-in.
    uint64_t G;
    X[0] = Eq[0] & S.P[0];
    asm("v_add_co_u32 %0, %1, %0, %2" : "+v"(X[0]), "=s"(G) : "v"(S.P[0]));
#pragma unroll
    for (int k = 1; k < KL; ++k) {
        X[k] = Eq[k] & S.P[k];
        asm("v_addc_co_u32 %0, %1, %0, %2, %1" : "+v"(X[k]), "+s"(G) : "v"(S.P[k]));
    }
    uint32_t all = X[0];
#pragma unroll
    for (int k = 1; k < KL; ++k) all &= X[k];
    const uint64_t Pr = __ballot(all == 0xffffffffu);
    const uint64_t B = G | Pr;
    uint64_t C = (G + B) ^ G ^ B;  // bit l = carry into lane l
    asm("v_addc_co_u32 %0, %1, %0, 0, %1" : "+v"(X[0]), "+s"(C));
#pragma unroll
    for (int k = 1; k < KL; ++k) asm("v_addc_co_u32 %0, %1, %0, 0, %1" : "+v"(X[k]), "+s"(C));
#pragma unroll
    for (int k = 0; k < KL; ++k) {
        Xh[k] = (X[k] ^ S.P[k]) | Eq[k];
        Ph[k] = S.M[k] | ~(Xh[k] | S.P[k]);
        Mh[k] = S.P[k] & Xh[k];
    }
    S.acc = wa_alignbit(S.M[0] | Xh[0], S.acc, 1);
    // Xs = Xv >> 1 across the wave; lane 63's top bit is Eq bit 2w (M bit 2w = 0: inserted +1)
    uint32_t nb = (uint32_t)__builtin_amdgcn_mov_dpp((int)Xv[0], 0x130 /* wave_shl:1 */, 0xf, 0xf, true);
    nb = lane == 63 ? (d[KL] >> t) : nb;
#pragma unroll
    for (int k = 0; k + 1 < KL; ++k) Xs[k] = wa_alignbit(Xv[k + 1], Xv[k], 1);
    Xs[KL - 1] = wa_alignbit(nb, Xv[KL - 1], 1);
#pragma unroll
    for (int k = 0; k < KL; ++k) {
        S.P[k] = Mh[k] | ~(Xs[k] | Ph[k]);
        S.M[k] = Ph[k] & Xs[k];
    }
}

// sum over band bits [0, kp) of (P - M), whole wave
template <int KL>
__device__ __forceinline__ int32_t wide_prefix(const WideState<KL> &S, uint32_t kp, uint32_t lane) {
    int32_t v = 0;
#pragma unroll
    for (int k = 0; k < KL; ++k) {
        const int32_t lo = (int32_t)kp - (int32_t)(32 * (KL * lane + k));
        const uint32_t mask = lo >= 32 ? 0xffffffffu : (lo <= 0 ? 0u : ((1u << lo) - 1));
        v += __builtin_popcount(S.P[k] & mask) - __builtin_popcount(S.M[k] & mask);
    }
    return (int32_t)wave_sum_u32((uint32_t)v);
}

template <int KL>
__device__ __forceinline__ void wide_load(uint32_t (&d)[KL + 1], const uint32_t *row_lane) {
    if constexpr (KL == 4) {
        const u32x4u v = *(const u32x4u *)row_lane;
        d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
        d[4] = row_lane[4];
    } else {
#pragma unroll
        for (int k = 0; k <= KL; ++k) d[k] = row_lane[k];
    }
}

// ED_w of one pair: the query side's match table `prow` ([n_sym][ndw], the query's length n) against stored trace
// j (length m) as the text, one wave; wave-uniform arguments. min(D_band, w + 1).
template <int KL>
__device__ __forceinline__ uint32_t wide_pair(const EdWideArgs &A, const uint32_t *prow, uint32_t n, uint64_t j,
                                              uint32_t m, uint32_t lane) {
    constexpr uint32_t W = 1024 * KL;
    const uint32_t w = A.w;
    uint32_t r = w + 1;
    const int64_t dd = (int64_t)m - (int64_t)n;
    if (dd > (int64_t)w || dd < -(int64_t)w) return r;
    if (n == 0 || m == 0) return n + m;
    // The query's match table through a buffer descriptor: per column the load's scalar offset
    // is (row byte offset of the candidate's symbol) + (band dword) * 4, the lane's part a
    // constant VGPR -- one s_add per column instead of a 64-bit address computation.
    const __amdgpu_buffer_rsrc_t rsrc = __builtin_amdgcn_make_buffer_rsrc(
        (void *)prow, (short)0, (int)(A.n_sym * A.ndw * 4), 0x00020000);
    const uint32_t voff = KL * lane * 4;
    // candidate's per-position row offsets: wave-uniform, read through the scalar cache
    typedef const uint32_t __attribute__((address_space(4))) *cptr;
    const uint64_t rb = __builtin_amdgcn_readfirstlane((uint32_t)A.rowb_off[j]) |
                        ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(A.rowb_off[j] >> 32)) << 32);
    const cptr rowb = (cptr)(const void *)(A.rowb + rb);
    WideState<KL> S;
#pragma unroll
    for (int k = 0; k < KL; ++k) {
        S.M[k] = (32 * (KL * lane + k) < W) ? 0xffffffffu : 0u;
        S.P[k] = ~S.M[k];
    }
    S.acc = 0;
    uint32_t T = W;
    // Eq dwords of column jj (1-based): row b_{jj}, dword (jj+31)>>5 + KL*lane, shift (jj-1)&31
    auto load_col = [&](uint32_t (&d)[KL + 1], uint32_t row_bytes, uint32_t jj) {
        const uint32_t so = row_bytes + ((jj + 31) >> 5) * 4;
        if constexpr (KL == 4) {
            const u32x4u v = __builtin_amdgcn_raw_buffer_load_b128(rsrc, voff, so, 0);
            d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
            d[4] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 16, so, 0);
        } else {
#pragma unroll
            for (int k = 0; k <= KL; ++k) d[k] = __builtin_amdgcn_raw_buffer_load_b32(rsrc, voff + 4 * k, so, 0);
        }
    };
    constexpr int D = 8;
    uint32_t cur[32], nxt[32];  // row offsets of this block's and the next block's columns
#pragma unroll
    for (int k = 0; k < 32; ++k) cur[k] = rowb[k];
    uint32_t ring[D][KL + 1];
#pragma unroll
    for (int u = 0; u < D; ++u) load_col(ring[u], cur[u], 1 + u);
    uint32_t j0 = 0;
    for (; j0 + 32 <= m; j0 += 32) {
#pragma unroll
        for (int k = 0; k < 32; ++k) nxt[k] = rowb[j0 + 32 + k];  // streams carry 2 spare blocks
#pragma unroll
        for (int t = 0; t < 32; ++t) {
            uint32_t dcur[KL + 1];
#pragma unroll
            for (int k = 0; k <= KL; ++k) dcur[k] = ring[t % D][k];
            load_col(ring[t % D], t + D < 32 ? cur[t + D] : nxt[t + D - 32], j0 + t + 1 + D);
            wide_column<KL>(S, dcur, t, lane);
        }
#pragma unroll
        for (int k = 0; k < 32; ++k) cur[k] = nxt[k];
        T += 32 - __builtin_popcount(__builtin_amdgcn_readfirstlane(S.acc));
        if (j0 + 32 == m) return min((uint32_t)((int32_t)T + wide_prefix<KL>(S, n + W - m, lane)), w + 1);
        uint32_t mc = 0;
#pragma unroll
        for (int k = 0; k < KL; ++k) mc += __builtin_popcount(S.M[k]);
        mc = wave_sum_u32(mc);
        if ((int32_t)T - (int32_t)mc > (int32_t)w) return r;  // band minimum > w: result w+1
    }
    // tail: fewer than 32 columns left, column m ends inside this block
    const uint32_t tail = m - j0;
    for (uint32_t t = 0; t < tail; ++t) {
        uint32_t dcur[KL + 1];
        load_col(dcur, rowb[j0 + t], j0 + t + 1);
        wide_column<KL>(S, dcur, t, lane);
    }
    const uint32_t acc0 = __builtin_amdgcn_readfirstlane(S.acc);
    const uint32_t Tj = T + tail - __builtin_popcount(acc0 >> (32 - tail));
    return min((uint32_t)((int32_t)Tj + wide_prefix<KL>(S, n + W - m, lane)), w + 1);
}

template <int KL>
__global__ __launch_bounds__(256) void k_ed_wide(EdWideArgs A) {
    const uint32_t nblk = gridDim.x, per_xcd = nblk / 8;
    const uint32_t lb = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    const uint32_t lwave = __builtin_amdgcn_readfirstlane(lb * 4 + (threadIdx.x >> 6));  // wave-uniform
    const uint32_t lane = threadIdx.x & 63;
    if (lwave >= A.n_waves) return;
    const uint64_t p = ((uint64_t)(lwave / 32) * A.n_shards + A.shard) * 32 + lwave % 32;
    if (p >= A.n_pairs) return;
    // p-th pair (i < j) of the upper triangle, row-major
    const uint64_t N = A.N;
    auto base = [&](uint64_t r) { return r * (2 * N - r - 1) / 2; };
    uint64_t i = (uint64_t)__builtin_amdgcn_readfirstlane(
        (uint32_t)floor(((2.0 * N - 1) - sqrt((2.0 * N - 1) * (2.0 * N - 1) - 8.0 * (double)p)) / 2));
    while (i > 0 && base(i) > p) --i;
    while (base(i + 1) <= p) ++i;
    const uint64_t j = __builtin_amdgcn_readfirstlane((uint32_t)(i + 1 + (p - base(i))));
    const uint32_t n = __builtin_amdgcn_readfirstlane((uint32_t)(A.off[i + 1] - A.off[i]));
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(A.off[j + 1] - A.off[j]));
    const uint32_t r = wide_pair<KL>(A, A.peq + (uint64_t)i * A.n_sym * A.ndw, n, j, m, lane);
    if (lane == 0) {
        wide_knn_insert(A.knn + i * A.k, A.k, ((uint64_t)r << 32) | j);
        wide_knn_insert(A.knn + j * A.k, A.k, ((uint64_t)r << 32) | i);
    }
}

// Single queries against the resident store (nmz_ed_plan_query_knn on a wide plan): wave (query q, stored trace j),
// the query's match table built for this call (qpeq: [n_q][qstride] dwords, rows over the store's alphabet; query
// symbols the store has never seen set bits in a row no stored trace names), results straight into the query's
// k-NN list. A query's waves are consecutive in the XCD-remapped order, so its table stays in one XCD's L2.
template <int KL>
__global__ __launch_bounds__(256) void k_ed_wide_query(EdWideArgs A, const uint32_t *__restrict__ qpeq,
                                                       uint64_t qstride, const uint32_t *__restrict__ qlen,
                                                       uint32_t n_q) {
    const uint32_t nblk = gridDim.x, per_xcd = nblk / 8;
    const uint32_t lb = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    const uint64_t lwave = __builtin_amdgcn_readfirstlane(lb * 4 + (threadIdx.x >> 6));
    const uint32_t lane = threadIdx.x & 63;
    if (lwave >= (uint64_t)n_q * A.N) return;
    const uint32_t q = __builtin_amdgcn_readfirstlane((uint32_t)(lwave / A.N));
    const uint64_t j = __builtin_amdgcn_readfirstlane((uint32_t)(lwave % A.N));
    const uint32_t n = __builtin_amdgcn_readfirstlane(qlen[q]);
    const uint32_t m = __builtin_amdgcn_readfirstlane((uint32_t)(A.off[j + 1] - A.off[j]));
    const uint32_t r = wide_pair<KL>(A, qpeq + (uint64_t)q * qstride, n, j, m, lane);
    if (lane == 0 && r <= A.w) wide_knn_insert(A.knn + (uint64_t)q * A.k, A.k, ((uint64_t)r << 32) | j);
}

// match bitmaps: peq[i][c][dword], bit (pos + 1 + OFF) of row sym[pos] for every position of trace i
__global__ void k_wide_peq_build(const uint16_t *__restrict__ sym, const uint64_t *__restrict__ off, uint32_t N,
                                 uint32_t n_sym, uint32_t ndw, uint32_t OFF, uint32_t *__restrict__ peq) {
    const uint64_t total = off[N];
    for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < total;
         t += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = N;  // trace: largest i with off[i] <= t
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) / 2;
            if (off[mid] <= t) lo = mid; else hi = mid;
        }
        const uint64_t pos = t - off[lo];
        const uint64_t bit = pos + 1 + OFF;
        atomicOr(&peq[((uint64_t)lo * n_sym + sym[t]) * ndw + (bit >> 5)], 1u << (bit & 31));
    }
}

bool ed_wide_supported(uint32_t band) { return band > 64 && band <= 8192; }
uint32_t ed_wide_template(uint32_t band) { return band <= 1024 ? 1024 : band <= 2048 ? 2048 : band <= 4096 ? 4096 : 8192; }

uint32_t ed_wide_ndw(uint32_t band, uint32_t max_len) {
    const uint32_t KL = band / 1024;
    return (max_len + band + 96) / 32 + 64 * KL + 16;
}

int ed_wide_build_peq(const uint16_t *d_sym, const uint64_t *d_off, uint32_t N, uint32_t n_sym, uint32_t ndw,
                      uint32_t band, uint32_t *d_peq, hipStream_t st) {
    NMZ_HIP(hipMemsetAsync(d_peq, 0, (size_t)N * n_sym * ndw * 4, st));
    hipLaunchKernelGGL(k_wide_peq_build, dim3(2048), dim3(256), 0, st, d_sym, d_off, N, n_sym, ndw, band + 31,
                       d_peq);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

int ed_wide_query_launch(const EdWideArgs &A, uint32_t band, const uint32_t *qpeq, uint64_t qstride,
                         const uint32_t *qlen, uint32_t n_q, hipStream_t st) {
    uint64_t blocks = ((uint64_t)n_q * A.N + 3) / 4;
    blocks = (blocks + 7) / 8 * 8;
    if (blocks == 0) return NMZ_OK;
    NMZ_CHECK(blocks < (1ULL << 30), "too many pairs for one launch");
    const dim3 g((unsigned)blocks), b(256);
    switch (band) {
        case 1024: hipLaunchKernelGGL(k_ed_wide_query<1>, g, b, 0, st, A, qpeq, qstride, qlen, n_q); break;
        case 2048: hipLaunchKernelGGL(k_ed_wide_query<2>, g, b, 0, st, A, qpeq, qstride, qlen, n_q); break;
        case 4096: hipLaunchKernelGGL(k_ed_wide_query<4>, g, b, 0, st, A, qpeq, qstride, qlen, n_q); break;
        case 8192: hipLaunchKernelGGL(k_ed_wide_query<8>, g, b, 0, st, A, qpeq, qstride, qlen, n_q); break;
        default: return fail(NMZ_EINVAL, "internal: band has no wide kernel");
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

int ed_wide_launch(const EdWideArgs &A, uint32_t band, hipStream_t st) {
    uint64_t blocks = (A.n_waves + 3) / 4;
    blocks = (blocks + 7) / 8 * 8;
    NMZ_CHECK(blocks < (1ULL << 30), "too many pairs for one launch");
    switch (band) {
        case 1024: hipLaunchKernelGGL(k_ed_wide<1>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
        case 2048: hipLaunchKernelGGL(k_ed_wide<2>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
        case 4096: hipLaunchKernelGGL(k_ed_wide<4>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
        case 8192: hipLaunchKernelGGL(k_ed_wide<8>, dim3((unsigned)blocks), dim3(256), 0, st, A); break;
        default: return fail(NMZ_EINVAL, "internal: band has no wide kernel");
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz
