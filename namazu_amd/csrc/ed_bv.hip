// K3b -- bit-parallel banded Levenshtein (Myers 1999 / Hyyro 2003, diagonal
// band) for the all-pairs k-NN search over event-hash traces.
//
// ED_w(a,b) = min(D_band(n,m), w+1) exactly as k_ed_tile / the oracle define
// it.  Any DP whose boundary values are upper bounds of
// the true Levenshtein values and finite outside the band gives a D' with
// Lev <= D' <= D_band on the band; both ends agree once clamped at w+1, so
// the band edges here carry +1 deltas (an upper bound) instead of +inf.
//
// Layout of one wave: 64 candidate traces b (one per lane) x 2 query traces
// a1, a2 (shared by the wave, held in LDS).  The query is the bit-vector
// "pattern": rows = query positions, columns = candidate positions.  Per
// column j a lane keeps the vertical deltas of the 2w+1 band rows
// r_j .. r_j+2w (r_j = j-w) as two bit-vectors P (+1) and M (-1) of KF
// 32-bit words; bit k <-> row r_j+k.  One column step is ~13 VALU ops per
// word instead of ~3 ops per DP cell: for w = 32 one step covers 65 cells.
//
//   Eq  = Peq_a[b_j] bits r_j..r_j+2w      (LDS; per-query match bitmaps)
//   Xv  = Eq | M
//   Xh  = (((Eq & P) + P) ^ P) | Eq
//   Ph  = M | ~(Xh | P)         Mh = P & Xh          (horizontal deltas)
//   Xs  = Xv >> 1                                    (band slides one row down)
//   P'  = Mh | ~(Xs | Ph)       M' = Ph & Xs         (+1 inserted at bit 2w)
//
// Query rows <= 0 are virtual rows with D(i,j) = j - i, a fixed point of the
// recurrence that reproduces row 0 (D(0,j) = j) and the +1 top boundary, so
// every column runs the same code.  The value of the band's top cell
// T_j = D(r_j, j) advances by vdelta + hdelta = 1 - ((M | Xh) & 1); the bits
// are shifted into an accumulator and popcounted once per 32 columns.
// Cut-off: D is non-decreasing along diagonals, so min(band at column j)
// never decreases; T_j - popcount(M) is a lower bound of it, and once it
// exceeds w the pair's result is w+1.
//
// Peq tables: per query, one bit row per symbol of the plan's alphabet
// (dense ids), 2 queries interleaved per dword ([symbol][dword][query]) so
// one ds_read_b64 returns a dword of both queries.  Candidate symbols are
// stored as that row's LDS byte offset (u16), one stream per trace.
// Compact tables (CMP, stores whose alphabet does not fit LDS): the streams
// hold dense symbol ids; a workgroup gives a row only to the distinct symbols
// of its two queries (row 0 = the zero row) and translates a candidate symbol
// through an LDS map id -> row byte offset (u16), one extra ds_read_u16 per
// column.  Exact: a symbol absent from both queries matches no query row.
//
// Band: the kernels compute the band of their template W (8, 16, 32, 64) and
// apply the requested w <= W at run time (length band, q-gram bound, cut-off,
// clamp): a path of cost c <= w never leaves the diagonals |i - j| <= c, so
// min(D_W, w + 1) = min(D_w, w + 1) (= min(Lev, w + 1)).
#include <type_traits>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

__device__ __forceinline__ uint32_t alignbit(uint32_t hi, uint32_t lo, uint32_t s) {
    return __builtin_amdgcn_alignbit(hi, lo, s);
}

__device__ __forceinline__ void bv_knn_insert(uint64_t *list, uint32_t k, uint64_t key) {
    if (key >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
    for (uint32_t s = 0; s < k; ++s) {
        const uint64_t old = atomicMin((unsigned long long *)&list[s], (unsigned long long)key);
        if (old == UINT64_MAX) return;
        key = old > key ? old : key;
    }
}

__device__ __forceinline__ void bv_knn_insert_wave(uint64_t *list, uint32_t k, uint64_t key, uint32_t lane) {
    for (uint32_t r = 0; r < k; ++r) {
        uint64_t best = key;
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) {
            const uint64_t o = __shfl_xor(best, off, 64);
            best = o < best ? o : best;
        }
        if (best == UINT64_MAX) return;
        if (best >= __hip_atomic_load(&list[k - 1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) return;
        if (lane == (uint32_t)__builtin_amdgcn_readfirstlane(__ffsll(__ballot(key == best)) - 1))
            bv_knn_insert(list, k, best);
        if (key == best) key = UINT64_MAX;
    }
}

template <int W>
struct BvShape {
    static constexpr int KF = (2 * W + 31) / 32;           // words holding band bits 0..2w-1
    static constexpr bool ELIDE = (2 * W == 32 * KF);       // insertion bit 2w in a word of its own
    static constexpr int ND = KF + 1;                       // dwords fetched per query per column
    static constexpr int OFF = W + 31;                      // Peq bit of query row i = i + OFF
    static constexpr uint32_t TOPMASK = ELIDE ? 0xffffffffu : ((1u << ((2 * W) & 31)) - 1);
};

// one query's column state
template <int KF>
struct BvState {
    uint32_t P[KF], M[KF];
    uint32_t acc;  // bit per column: (M | Xh) & 1  (= 1 - increment of T)
    uint32_t T;    // T at the start of the current 32-column block
};

template <int W, int t>
__device__ __forceinline__ void bv_column(BvState<BvShape<W>::KF> &S, const uint32_t (&d)[BvShape<W>::ND]) {
    using SH = BvShape<W>;
    constexpr int KF = SH::KF;
    uint32_t Eq[KF], Xv[KF], Xh[KF], Ph[KF], Mh[KF];
#pragma unroll
    for (int k = 0; k < KF; ++k) Eq[k] = t == 0 ? d[k] : alignbit(d[k + 1], d[k], t);
#pragma unroll
    for (int k = 0; k < KF; ++k) Xv[k] = Eq[k] | S.M[k];
    // X = (Eq & P) + P over KF words
    if constexpr (KF == 1) {
        const uint32_t X = (Eq[0] & S.P[0]) + S.P[0];
        Xh[0] = (X ^ S.P[0]) | Eq[0];
    } else if constexpr (KF == 2) {
        const uint64_t p = ((uint64_t)S.P[1] << 32) | S.P[0];
        const uint64_t e = ((uint64_t)(Eq[1] & S.P[1]) << 32) | (Eq[0] & S.P[0]);
        const uint64_t X = e + p;
        Xh[0] = ((uint32_t)X ^ S.P[0]) | Eq[0];
        Xh[1] = ((uint32_t)(X >> 32) ^ S.P[1]) | Eq[1];
    } else {
        static_assert(KF == 4, "KF in {1, 2, 4} (w <= 64)");
        const uint64_t p0 = ((uint64_t)S.P[1] << 32) | S.P[0], p1 = ((uint64_t)S.P[3] << 32) | S.P[2];
        const uint64_t e0 = ((uint64_t)(Eq[1] & S.P[1]) << 32) | (Eq[0] & S.P[0]);
        const uint64_t e1 = ((uint64_t)(Eq[3] & S.P[3]) << 32) | (Eq[2] & S.P[2]);
        const uint64_t X0 = e0 + p0;
        const uint64_t X1 = e1 + p1 + (uint64_t)(X0 < p0);
        Xh[0] = ((uint32_t)X0 ^ S.P[0]) | Eq[0];
        Xh[1] = ((uint32_t)(X0 >> 32) ^ S.P[1]) | Eq[1];
        Xh[2] = ((uint32_t)X1 ^ S.P[2]) | Eq[2];
        Xh[3] = ((uint32_t)(X1 >> 32) ^ S.P[3]) | Eq[3];
    }
#pragma unroll
    for (int k = 0; k < KF; ++k) {
        Ph[k] = S.M[k] | ~(Xh[k] | S.P[k]);
        Mh[k] = S.P[k] & Xh[k];
    }
    S.acc = alignbit(S.M[0] | Xh[0], S.acc, 1);
    uint32_t Xs[KF];
#pragma unroll
    for (int k = 0; k + 1 < KF; ++k) Xs[k] = alignbit(Xv[k + 1], Xv[k], 1);
    if constexpr (SH::ELIDE) {
        // bit 2w-1 of Xs = Xv bit 2w = Eq bit 2w (M bit 2w is 0: inserted +1)
        Xs[KF - 1] = alignbit(d[KF] >> t, Xv[KF - 1], 1);
    } else {
        Xs[KF - 1] = Xv[KF - 1] >> 1;
    }
#pragma unroll
    for (int k = 0; k < KF; ++k) {
        S.P[k] = Mh[k] | ~(Xs[k] | Ph[k]);
        S.M[k] = Ph[k] & Xs[k];
    }
    if constexpr (!SH::ELIDE) {
        constexpr uint32_t ins = 1u << ((2 * W) & 31);
        S.P[KF - 1] |= ins;
        S.M[KF - 1] &= ~ins;
    }
}

// D(n, m) once column m = j is done: T_j + sum of the first k' vertical deltas
template <int W>
__device__ __forceinline__ uint32_t bv_extract(const BvState<BvShape<W>::KF> &S, uint32_t Tj, uint32_t kp) {
    int32_t v = (int32_t)Tj;
#pragma unroll
    for (int k = 0; k < BvShape<W>::KF; ++k) {
        const int32_t lo = (int32_t)kp - 32 * k;
        const uint32_t mask = lo >= 32 ? 0xffffffffu : (lo <= 0 ? 0u : ((1u << lo) - 1));
        v += __builtin_popcount(S.P[k] & mask) - __builtin_popcount(S.M[k] & mask);
    }
    return (uint32_t)v;
}

template <int W>
__device__ __forceinline__ void bv_init(BvState<BvShape<W>::KF> &S) {
    // column 0: rows r_1+k (r_1 = 1-w): k < w are rows <= 0 (delta -1), k >= w rows >= 1 (+1)
#pragma unroll
    for (int k = 0; k < BvShape<W>::KF; ++k) {
        uint32_t mm = 0, pp = 0;
        for (int b = 0; b < 32; ++b) {
            const int bit = 32 * k + b;
            if (bit < W) mm |= 1u << b;
            else if (bit <= 2 * W) pp |= 1u << b;
        }
        S.M[k] = mm;
        S.P[k] = pp;
    }
    S.acc = 0;
    S.T = W;
}

template <int W>
__device__ __forceinline__ uint32_t bv_lower_bound(const BvState<BvShape<W>::KF> &S, uint32_t Tj) {
    int32_t v = (int32_t)Tj;
#pragma unroll
    for (int k = 0; k < BvShape<W>::KF; ++k)
        v -= __builtin_popcount(k == BvShape<W>::KF - 1 ? (S.M[k] & BvShape<W>::TOPMASK) : S.M[k]);
    return (uint32_t)(v < 0 ? 0 : v);
}

template <int W, int t, bool SLOW>
__device__ __forceinline__ void bv_step2(BvState<BvShape<W>::KF> &S1, BvState<BvShape<W>::KF> &S2,
                                         const uint32_t *peq_bytes, uint32_t addr, uint32_t j, uint32_t m,
                                         uint32_t n1, uint32_t n2, bool &run1, bool &run2, uint32_t &r1,
                                         uint32_t &r2, uint32_t w1) {
    using SH = BvShape<W>;
    const uint2 *pp = (const uint2 *)((const char *)peq_bytes + addr);
    uint32_t d1[SH::ND], d2[SH::ND];
#pragma unroll
    for (int k = 0; k < SH::ND; ++k) {
        const uint2 x = pp[k];
        d1[k] = x.x;
        d2[k] = x.y;
    }
    bv_column<W, t>(S1, d1);
    bv_column<W, t>(S2, d2);
    if constexpr (SLOW) {
        if (j == m) {
            if (run1) {
                const uint32_t Tj = S1.T + (t + 1) - __builtin_popcount(S1.acc >> (31 - t));
                r1 = min(bv_extract<W>(S1, Tj, n1 + W - m), w1);
                run1 = false;
            }
            if (run2) {
                const uint32_t Tj = S2.T + (t + 1) - __builtin_popcount(S2.acc >> (31 - t));
                r2 = min(bv_extract<W>(S2, Tj, n2 + W - m), w1);
                run2 = false;
            }
        }
    }
}

// one query of the interleaved pair tables (addr already + 4 * query slot): its dwords are 8 bytes apart
template <int W, int t, bool SLOW>
__device__ __forceinline__ void bv_step1(BvState<BvShape<W>::KF> &S, const uint32_t *peq_bytes, uint32_t addr,
                                         uint32_t j, uint32_t m, uint32_t n, bool &run, uint32_t &r, uint32_t w1) {
    using SH = BvShape<W>;
    const uint32_t *pp = (const uint32_t *)((const char *)peq_bytes + addr);
    uint32_t d[SH::ND];
#pragma unroll
    for (int k = 0; k < SH::ND; ++k) d[k] = pp[2 * k];
    bv_column<W, t>(S, d);
    if constexpr (SLOW) {
        if (j == m && run) {
            const uint32_t Tj = S.T + (t + 1) - __builtin_popcount(S.acc >> (31 - t));
            r = min(bv_extract<W>(S, Tj, n + W - m), w1);
            run = false;
        }
    }
}

template <int W, bool CMP, bool SLOW, int t = 0>
__device__ __forceinline__ void bv_block1(BvState<BvShape<W>::KF> &S, const uint32_t *peq, const uint16_t *rmap,
                                          const uint32_t (&sym)[16], uint32_t base, uint32_t j0, uint32_t m,
                                          uint32_t n, bool &run, uint32_t &r, uint32_t w1) {
    if constexpr (t < 32) {
        const uint32_t w = sym[t / 2];
        const uint32_t s = (t & 1) ? (w >> 16) : (w & 0xffffu);
        const uint32_t addr = (CMP ? (uint32_t)rmap[s] : s) + base;
        bv_step1<W, t, SLOW>(S, peq, addr, j0 + t + 1, m, n, run, r, w1);
        bv_block1<W, CMP, SLOW, t + 1>(S, peq, rmap, sym, base, j0, m, n, run, r, w1);
    }
}

// The one-query block with its Peq reads issued NMZ_ED_PF columns ahead. Column t's rows depend only on the block's
// symbols, but bv_block1 reads each column's rows one column before its step, so a chain-bound wave (a sparse
// shard's DP: ~1 wave per SIMD) waits most of an LDS round trip in every column. Here a compact store's symbols are
// mapped to row offsets once per block (sym is overwritten: the caller replaces it with the next block), then a ring
// of PF columns' rows stays in flight ahead of the step. Under the kernel's 96-VGPR cap (5 waves/SIMD) PF = 3 adds no
// spill to the direct-table kernels (PF 4: 14 more scratch ops outside the block, PF 6: 6 inside it); with compact
// tables the in-place row mapping spills (47 scratch ops at PF 3 against 14), so those keep bv_block1 unless
// NMZ_ED_PF_CMP=1 (an A/B build).
#ifndef NMZ_ED_PF
#define NMZ_ED_PF 3
#endif
#ifndef NMZ_ED_PF_CMP
#define NMZ_ED_PF_CMP 0
#endif
#ifndef NMZ_ED_PF_SB
#define NMZ_ED_PF_SB 0
#endif
#if NMZ_ED_PF > 0
template <int W>
__device__ __forceinline__ void bv_fetch1(uint32_t (&d)[BvShape<W>::ND], const uint32_t *peq_bytes, uint32_t addr) {
    const uint32_t *pp = (const uint32_t *)((const char *)peq_bytes + addr);
#pragma unroll
    for (int k = 0; k < BvShape<W>::ND; ++k) d[k] = pp[2 * k];
}

template <int W, int PF, bool SLOW, int t>
__device__ __forceinline__ void bv_cols1(BvState<BvShape<W>::KF> &S, uint32_t (&ring)[PF][BvShape<W>::ND],
                                         const uint32_t *peq, const uint32_t (&sym)[16], uint32_t base, uint32_t j0,
                                         uint32_t m, uint32_t n, bool &run, uint32_t &r, uint32_t w1) {
    if constexpr (t < 32) {
        using SH = BvShape<W>;
        uint32_t d[SH::ND];
#pragma unroll
        for (int k = 0; k < SH::ND; ++k) d[k] = ring[t % PF][k];
        if constexpr (t + PF < 32) {
            const uint32_t w = sym[(t + PF) / 2];
            bv_fetch1<W>(ring[t % PF], peq, (((t + PF) & 1) ? (w >> 16) : (w & 0xffffu)) + base);
#if NMZ_ED_PF_SB
            __builtin_amdgcn_sched_barrier(0);  // keep the reads here (the scheduler sinks them to their use)
#endif
        }
        bv_column<W, t>(S, d);
        if constexpr (SLOW) {
            if (j0 + t + 1 == m && run) {
                const uint32_t Tj = S.T + (t + 1) - __builtin_popcount(S.acc >> (31 - t));
                r = min(bv_extract<W>(S, Tj, n + W - m), w1);
                run = false;
            }
        }
        bv_cols1<W, PF, SLOW, t + 1>(S, ring, peq, sym, base, j0, m, n, run, r, w1);
    }
}

template <int W, bool CMP, bool SLOW>
__device__ __forceinline__ void bv_block1_pf(BvState<BvShape<W>::KF> &S, const uint32_t *peq, const uint16_t *rmap,
                                             uint32_t (&sym)[16], uint32_t base, uint32_t j0, uint32_t m, uint32_t n,
                                             bool &run, uint32_t &r, uint32_t w1) {
    constexpr int PF = NMZ_ED_PF;
    if constexpr (CMP) {
#pragma unroll
        for (int i = 0; i < 16; ++i) sym[i] = (uint32_t)rmap[sym[i] & 0xffffu] | ((uint32_t)rmap[sym[i] >> 16] << 16);
    }
    uint32_t ring[PF][BvShape<W>::ND];
#pragma unroll
    for (int t = 0; t < PF; ++t) {
        const uint32_t w = sym[t / 2];
        bv_fetch1<W>(ring[t], peq, ((t & 1) ? (w >> 16) : (w & 0xffffu)) + base);
    }
    bv_cols1<W, PF, SLOW, 0>(S, ring, peq, sym, base, j0, m, n, run, r, w1);
}
#endif

// The two-query block (bv_dp_run's lanes: both queries of the pair per candidate) with its Peq reads issued
// NMZ_ED_PF2 columns ahead (0 = bv_block, which reads each column one column before its step). The
// paired loop runs at 5 waves per SIMD, so other waves cover most of the LDS latency: configs[2] clustered leg
// 73.5 -> 71.5 ms at 2 (r06z, 2 runs each), 74.1 ms at 3 (50 more scratch ops outside the block). Compact tables
// map each symbol to its row offset PF columns before that column's read (a ring of PF offsets; mapping the whole
// block in place spilled 26 scratch ops into the block): configs[2] 3,572-symbol store 81.0 -> 75.5 ms (r06ac).
// NMZ_ED_PF2_CMP=0 keeps bv_block for compact tables (an A/B build).
#ifndef NMZ_ED_PF2
#define NMZ_ED_PF2 2
#endif
#ifndef NMZ_ED_PF2_CMP
#define NMZ_ED_PF2_CMP 1
#endif
#if NMZ_ED_PF2 > 0
template <int W>
__device__ __forceinline__ void bv_fetch2(uint2 (&d)[BvShape<W>::ND], const uint32_t *peq_bytes, uint32_t addr) {
    const uint2 *pp = (const uint2 *)((const char *)peq_bytes + addr);
#pragma unroll
    for (int k = 0; k < BvShape<W>::ND; ++k) d[k] = pp[k];
}

template <int t>
__device__ __forceinline__ uint32_t bv_sym_at(const uint32_t (&sym)[16]) {
    const uint32_t w = sym[t / 2];
    return (t & 1) ? (w >> 16) : (w & 0xffffu);
}

// the first PF columns' reads (and, compact tables, the next PF columns' row offsets)
template <int W, bool CMP, int PF, int t>
__device__ __forceinline__ void bv_block_pf_pro(uint2 (&ring)[PF][BvShape<W>::ND], uint32_t (&ra)[PF],
                                                const uint32_t *peq, const uint16_t *rmap, const uint32_t (&sym)[16],
                                                uint32_t base) {
    if constexpr (t < PF) {
        const uint32_t s = bv_sym_at<t>(sym);
        bv_fetch2<W>(ring[t], peq, (CMP ? (uint32_t)rmap[s] : s) + base);
        if constexpr (CMP) ra[t] = rmap[bv_sym_at<t + PF>(sym)];
        bv_block_pf_pro<W, CMP, PF, t + 1>(ring, ra, peq, rmap, sym, base);
    }
}

// (compact tables: ra holds the row offsets of the next PF columns to fetch, mapped PF columns before their fetch)
template <int W, bool CMP, int PF, bool SLOW, int t>
__device__ __forceinline__ void bv_cols2(BvState<BvShape<W>::KF> &S1, BvState<BvShape<W>::KF> &S2,
                                         uint2 (&ring)[PF][BvShape<W>::ND], uint32_t (&ra)[PF], const uint32_t *peq,
                                         const uint16_t *rmap, const uint32_t (&sym)[16], uint32_t base, uint32_t j0,
                                         uint32_t m, uint32_t n1, uint32_t n2, bool &run1, bool &run2, uint32_t &r1,
                                         uint32_t &r2, uint32_t w1) {
    if constexpr (t < 32) {
        using SH = BvShape<W>;
        uint32_t d1[SH::ND], d2[SH::ND];
#pragma unroll
        for (int k = 0; k < SH::ND; ++k) {
            d1[k] = ring[t % PF][k].x;
            d2[k] = ring[t % PF][k].y;
        }
        if constexpr (t + PF < 32) {
            bv_fetch2<W>(ring[t % PF], peq, (CMP ? ra[t % PF] : bv_sym_at<t + PF>(sym)) + base);
            if constexpr (CMP && t + 2 * PF < 32) ra[t % PF] = rmap[bv_sym_at<t + 2 * PF>(sym)];
        }
        bv_column<W, t>(S1, d1);
        bv_column<W, t>(S2, d2);
        if constexpr (SLOW) {
            if (j0 + t + 1 == m) {
                if (run1) {
                    const uint32_t Tj = S1.T + (t + 1) - __builtin_popcount(S1.acc >> (31 - t));
                    r1 = min(bv_extract<W>(S1, Tj, n1 + W - m), w1);
                    run1 = false;
                }
                if (run2) {
                    const uint32_t Tj = S2.T + (t + 1) - __builtin_popcount(S2.acc >> (31 - t));
                    r2 = min(bv_extract<W>(S2, Tj, n2 + W - m), w1);
                    run2 = false;
                }
            }
        }
        bv_cols2<W, CMP, PF, SLOW, t + 1>(S1, S2, ring, ra, peq, rmap, sym, base, j0, m, n1, n2, run1, run2, r1, r2,
                                          w1);
    }
}

template <int W, bool CMP, bool SLOW>
__device__ __forceinline__ void bv_block_pf(BvState<BvShape<W>::KF> &S1, BvState<BvShape<W>::KF> &S2,
                                            const uint32_t *peq, const uint16_t *rmap, const uint32_t (&sym)[16],
                                            uint32_t base, uint32_t j0, uint32_t m, uint32_t n1, uint32_t n2,
                                            bool &run1, bool &run2, uint32_t &r1, uint32_t &r2, uint32_t w1) {
    constexpr int PF = NMZ_ED_PF2;
    uint2 ring[PF][BvShape<W>::ND];
    uint32_t ra[PF];
    bv_block_pf_pro<W, CMP, PF, 0>(ring, ra, peq, rmap, sym, base);
    bv_cols2<W, CMP, PF, SLOW, 0>(S1, S2, ring, ra, peq, rmap, sym, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
}
#endif

// rmap: the compact tables' map symbol id -> row byte offset (LDS, CMP only)
template <int W, bool CMP, bool SLOW, int t = 0>
__device__ __forceinline__ void bv_block(BvState<BvShape<W>::KF> &S1, BvState<BvShape<W>::KF> &S2,
                                         const uint32_t *peq, const uint16_t *rmap, const uint32_t (&sym)[16],
                                         uint32_t base, uint32_t j0, uint32_t m, uint32_t n1, uint32_t n2, bool &run1,
                                         bool &run2, uint32_t &r1, uint32_t &r2, uint32_t w1) {
    if constexpr (t < 32) {
        const uint32_t w = sym[t / 2];
        const uint32_t s = (t & 1) ? (w >> 16) : (w & 0xffffu);
        const uint32_t addr = (CMP ? (uint32_t)rmap[s] : s) + base;
        bv_step2<W, t, SLOW>(S1, S2, peq, addr, j0 + t + 1, m, n1, n2, run1, run2, r1, r2, w1);
        bv_block<W, CMP, SLOW, t + 1>(S1, S2, peq, rmap, sym, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
    }
}

// The Peq rows of a workgroup's one or two queries (a1, n1 -> slot 0; a2, n2 -> slot 1) into the zeroed LDS
// tables: bit (i + 1 + OFF) of the row of the query's symbol i. Stream value 0xffff (a query symbol the store
// lacks) sets nothing. CMP: stream values are symbol ids; each distinct id first claims a row (atomicOr on a
// claim bitmap, row 0 stays the zero row) and rmap[id] = its byte offset; otherwise the values are the rows'
// byte offsets already.
template <int W, bool CMP>
__device__ __forceinline__ void bv_peq_build(uint32_t *peq, uint32_t rmap_dw, uint32_t claim_dw, uint32_t row_bytes,
                                             uint32_t *rows, const uint16_t *a1, uint32_t n1, const uint16_t *a2,
                                             uint32_t n2) {
    using SH = BvShape<W>;
    uint16_t *rmap = (uint16_t *)(peq + rmap_dw);
    if constexpr (CMP) {
        uint32_t *claim = peq + claim_dw;
        for (uint32_t q = 0; q < 2; ++q) {
            const uint16_t *a = q ? a2 : a1;
            const uint32_t n = q ? n2 : n1;
            for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
                const uint32_t s = a[i];
                if (s == 0xffffu) continue;
                const uint32_t bit = 1u << (s & 31);
                if (!(atomicOr(&claim[s >> 5], bit) & bit)) rmap[s] = (uint16_t)((atomicAdd(rows, 1u) + 1u) * row_bytes);
            }
        }
        __syncthreads();
    }
    for (uint32_t q = 0; q < 2; ++q) {
        const uint16_t *a = q ? a2 : a1;
        const uint32_t n = q ? n2 : n1;
        for (uint32_t i = threadIdx.x; i < n; i += blockDim.x) {
            const uint32_t s = a[i];
            if (s == 0xffffu) continue;
            const uint32_t off = CMP ? (uint32_t)rmap[s] : s;
            const uint32_t p = i + 1 + SH::OFF;
            atomicOr(&peq[off / 4 + (p >> 5) * 2 + q], 1u << (p & 31));
        }
    }
}

// ---------------------------------------------------------------------------
// k_ed_bv: the column step above with lane refill.  A workgroup owns 2 query
// traces and a pool of up to ED_BV_POOL candidate traces; each lane works
// on one candidate at a time and, when both of its pairs are finished
// (extracted or cut off), publishes them and takes the next candidate from
// the workgroup's LDS counter, restarting at column 1 in the next 32-column
// block (lanes may be at different columns; the in-block shift t stays
// wave-uniform because restarts happen on block boundaries).  A wave stops
// when the pool is empty and its lanes are idle, so its cost follows the
// mean cut-off column of its pairs instead of the maximum over 64 of them.
// Candidate streams are per trace ([pos] u16 Peq-row byte offsets, padded to
// whole 32-position blocks plus one spare block); the query's Peq rows are
// built from the same streams.
// ---------------------------------------------------------------------------
// publish the pairs of the lanes with `fin` set: candidate lists per lane
// (distinct lists), query lists wave-reduced (the 2 query lists are shared by
// every lane of the workgroup; per-lane atomics on them serialize in L2)
// Only results within the band are listed: every other pair's result is w + 1, and k_knn_fill completes the lists
// with (w + 1, smallest ids not listed) after the search, so the bulk of the pairs (cut off, out of the length band
// or settled by the q-gram bound) publish nothing and cost no global atomics.
__device__ __forceinline__ void bv_publish(const EdBvArgs &A, bool fin, uint32_t j, uint32_t q1, uint32_t q2,
                                            bool v2, uint32_t r1, uint32_t r2, uint32_t lane, uint32_t w,
                                            uint32_t &in_band) {
    const bool b1 = fin && r1 <= w, b2 = fin && v2 && r2 <= w;
    in_band += (uint32_t)b1 + (uint32_t)b2;
#ifdef NMZ_ABL_PUBLISH
    return;  // timing only: results not listed
#endif
    if (b1) bv_knn_insert(A.knn + (uint64_t)j * A.k, A.k, ((uint64_t)r1 << 32) | q1);
    if (b2) bv_knn_insert(A.knn + (uint64_t)j * A.k, A.k, ((uint64_t)r2 << 32) | q2);
    if (__any(b1)) bv_knn_insert_wave(A.knn + (uint64_t)q1 * A.k, A.k, b1 ? (((uint64_t)r1 << 32) | j) : UINT64_MAX, lane);
    if (__any(b2)) bv_knn_insert_wave(A.knn + (uint64_t)q2 * A.k, A.k, b2 ? (((uint64_t)r2 << 32) | j) : UINT64_MAX, lane);
}

__device__ __forceinline__ void bv_load_block(uint32_t (&dst)[16], const uint16_t *stream, uint32_t blk) {
    const uint4 *p = (const uint4 *)(stream + (uint64_t)blk * 32);
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const uint4 v = p[r];
        dst[4 * r] = v.x; dst[4 * r + 1] = v.y; dst[4 * r + 2] = v.z; dst[4 * r + 3] = v.w;
    }
}

// ---------------------------------------------------------------------------
// q-gram filter (nmz_internal.h ED_QG_*): bucket of the adjacent pair (x, y) of stream values (Peq-row byte
// offsets, i.e. dense symbol ids; 0xffff for a query symbol the store lacks, which merges such symbols -- a
// valid coarsening). Profiles are built once per plan; a lane compares its candidate's profile with the
// workgroup's query profiles by v_sad_u8 (|a - b| summed over 4 packed counts) before any DP.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t qg_bucket(uint32_t x, uint32_t y) {
    uint32_t h = x * 0x9E3779B1u + y * 0x85EBCA77u;
    h ^= h >> 15;
    h *= 0x2C1B3C6Du;
    return h >> (32 - 7);  // ED_QG_BUCKETS = 128
}

// one workgroup per trace: bigram counts in LDS, saturated at 255 and packed 4 per dword
__global__ __launch_bounds__(256) void k_ed_qgram_profile(const uint16_t *__restrict__ bs,
                                                          const uint64_t *__restrict__ soff,
                                                          const uint32_t *__restrict__ len, uint32_t *__restrict__ prof) {
    __shared__ uint32_t hist[ED_QG_BUCKETS];
    const uint32_t i = blockIdx.x;
    if (threadIdx.x < ED_QG_BUCKETS) hist[threadIdx.x] = 0;
    __syncthreads();
    const uint16_t *a = bs + soff[i];
    const uint32_t n = len[i];
    for (uint32_t t = threadIdx.x; t + 1 < n; t += 256) atomicAdd(&hist[qg_bucket(a[t], a[t + 1])], 1u);
    __syncthreads();
    if (threadIdx.x < ED_QG_DW) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= min(hist[4 * threadIdx.x + b], 255u) << (8 * b);
        prof[(uint64_t)i * ED_QG_DW + threadIdx.x] = w;
    }
}

int ed_qgram_profiles(const uint16_t *bs, const uint64_t *soff, const uint32_t *len, uint32_t N, uint32_t *prof,
                      hipStream_t st) {
    if (N == 0) return NMZ_OK;
    hipLaunchKernelGGL(k_ed_qgram_profile, dim3(N), dim3(256), 0, st, bs, soff, len, prof);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// L1 distance of a candidate's profile (global) to the two query profiles (LDS, 16-byte aligned)
__device__ __forceinline__ void qg_l1x2(const uint4 *__restrict__ cp, const uint4 *qp1, const uint4 *qp2,
                                        uint32_t &s1, uint32_t &s2) {
    s1 = 0;
    s2 = 0;
#pragma unroll
    for (int r = 0; r < (int)ED_QG_DW / 4; ++r) {
        const uint4 c = cp[r], a = qp1[r], b = qp2[r];
        s1 = __builtin_amdgcn_sad_u8(c.x, a.x, s1);
        s1 = __builtin_amdgcn_sad_u8(c.y, a.y, s1);
        s1 = __builtin_amdgcn_sad_u8(c.z, a.z, s1);
        s1 = __builtin_amdgcn_sad_u8(c.w, a.w, s1);
        s2 = __builtin_amdgcn_sad_u8(c.x, b.x, s2);
        s2 = __builtin_amdgcn_sad_u8(c.y, b.y, s2);
        s2 = __builtin_amdgcn_sad_u8(c.z, b.z, s2);
        s2 = __builtin_amdgcn_sad_u8(c.w, b.w, s2);
    }
}

#ifndef NMZ_ED_DP_MONO
#define NMZ_ED_DP_MONO 1
#endif

// Occupancy: 5 waves/SIMD (<= 96 VGPRs; the compiler spills 6 VGPRs outside the 32-column block). configs[2]
// clustered, 100k x 2,048: 1.509 s at the unconstrained 100 VGPRs (4 waves), 1.487 s at 5, 1.667 s at 6 (31
// spills, some in the block refill path). NMZ_ED_BV_WAVES overrides for A/B builds.
#ifndef NMZ_ED_BV_WAVES
#define NMZ_ED_BV_WAVES 5
#endif
// W = 64 (4 state words per query) at 4 waves/SIMD (128 VGPRs): at 5 it spilled 168 bytes per lane
#if NMZ_ED_BV_WAVES > 0
#define NMZ_ED_BV_ATTR \
    __attribute__((amdgpu_waves_per_eu(W == 64 ? 4 : NMZ_ED_BV_WAVES, W == 64 ? 4 : NMZ_ED_BV_WAVES)))
#else
#define NMZ_ED_BV_ATTR
#endif

// wave-reduce the work counters and add them to this workgroup's stripe of counters[] (nmz_ed_plan_counters)
__device__ __forceinline__ void bv_flush_counters(uint64_t *counters, uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                                  uint32_t c4, uint32_t c5) {
    if (!counters) return;
    uint64_t c[ED_BV_NCOUNTERS] = {c0, c1, c2, c3, c4, c5};
#pragma unroll
    for (int i = 0; i < ED_BV_NCOUNTERS; ++i) {
#pragma unroll
        for (int off = 32; off >= 1; off >>= 1) c[i] += __shfl_xor(c[i], off, 64);
    }
    if ((threadIdx.x & 63) == 0) {
        uint64_t *line = counters + (blockIdx.x % ED_CNT_STRIPES) * ED_CNT_LINE;
#pragma unroll
        for (int i = 0; i < ED_BV_NCOUNTERS; ++i)
            if (c[i]) atomicAdd((unsigned long long *)&line[i], (unsigned long long)c[i]);
    }
}

// The DP loop of a workgroup whose 2 queries' Peq tables are in LDS: `ns` entries (candidate j, run1, run2 --
// the pairs that need a DP, from fetch(idx, j, run1, run2)) drawn by the lanes through the LDS counter pool_next
// (which must start at 256: entries 0..255 are pre-assigned), each run to extraction or cut-off, the in-band
// results listed (bv_publish). Work counters are accumulated into the caller's registers.
template <int W, bool CMP, class Fetch>
__device__ __forceinline__ void bv_dp_run(const EdBvArgs &A, const uint32_t *peq, uint32_t &pool_next, uint32_t ns,
                                          uint32_t q1, uint32_t q2, uint32_t n1, uint32_t n2, bool has2, Fetch fetch,
                                          uint32_t &c_dp_pairs, uint32_t &c_in_band, uint32_t &c_blocks,
                                          uint32_t &c_dp_cand, uint32_t &c_live) {
    using SH = BvShape<W>;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = A.w, w1 = A.w + 1;
    const uint16_t *rmap = (const uint16_t *)(peq + A.rmap_dw);
    // lane state
    uint32_t j = 0, m = 0, r1 = w1, r2 = w1, kb0 = 0;
    bool run1 = false, run2 = false, active = false, v2 = false;
    const uint16_t *stream = A.bsym;
    BvState<SH::KF> S1, S2;
    uint32_t cur[16], nxt[16];
    uint32_t idx = threadIdx.x;  // the first 256 entries are pre-assigned
    uint32_t kb = 0;
    bool need = ns > 0;
    bool first = true;
    while (ns > 0) {
        // ---- (re)assign survivors to lanes that need one ----
        const uint64_t want = __ballot(need);
        if (want != 0) {
            if (!first) {
                const uint32_t cnt = __popcll(want);
                uint32_t base_idx = 0;
                if (lane == (uint32_t)(__ffsll((unsigned long long)want) - 1)) base_idx = atomicAdd(&pool_next, cnt);
                base_idx = __shfl(base_idx, __ffsll((unsigned long long)want) - 1, 64);
                if (need) idx = base_idx + __popcll(want & ((1ull << lane) - 1));
            }
            first = false;
            if (need) {
                need = false;
                if (idx >= ns) {
                    active = false;
                    stream = A.bsym;  // idle lanes keep reading a valid stream (results unused)
                    bv_load_block(cur, stream, 0);
                } else {
                    fetch(idx, j, run1, run2);
                    m = A.len[j];
                    stream = A.bsym + A.soff[j];
                    v2 = has2 && j > q2;
                    r1 = w1;
                    r2 = w1;
                    active = true;
                    c_dp_cand += 1;
                    c_dp_pairs += (uint32_t)run1 + (uint32_t)run2;
                    kb0 = kb;
                    bv_init<W>(S1);
                    bv_init<W>(S2);
                    bv_load_block(cur, stream, 0);
                }
            }
        }
        if (!__any(active)) break;
        c_blocks += (uint32_t)active;
        c_live += active ? (uint32_t)run1 + (uint32_t)run2 : 0u;
        // ---- one 32-column block ----
        const uint32_t lkb = active ? kb - kb0 : 0;
        bv_load_block(nxt, stream, lkb + 1);  // streams carry one spare block
        const uint32_t j0 = 32 * lkb;
        const uint32_t base = (lkb + 1) * 8;
        const bool here = active && (run1 || run2) && m > j0 && m <= j0 + 32;
#if NMZ_ED_PF2 > 0
        if constexpr (!CMP || NMZ_ED_PF2_CMP) {
            if (__any(here)) {
                bv_block_pf<W, CMP, true>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            } else {
                bv_block_pf<W, CMP, false>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            }
        } else
#endif
        {
            if (__any(here)) {
                bv_block<W, CMP, true>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            } else {
                bv_block<W, CMP, false>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            }
        }
        S1.T += 32 - __builtin_popcount(S1.acc);
        S2.T += 32 - __builtin_popcount(S2.acc);
        if (run1 && bv_lower_bound<W>(S1, S1.T) > w) run1 = false;
        if (run2 && bv_lower_bound<W>(S2, S2.T) > w) run2 = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[r] = nxt[r];
        ++kb;
        const bool fin = active && !run1 && !run2;
        if (__any(fin)) bv_publish(A, fin, j, q1, q2, v2, r1, r2, lane, w, c_in_band);
        if (fin) {
            active = false;
            need = true;
        }
    }
}

// An item of at most 128 entries (a sparse search: a query pair with a few DP candidates): lane 2e + s runs the
// single pair (query s of the pair, entry e's candidate) when entry e needs it, one query state per lane instead of
// two. A lane of the paired loop above steps both queries for every candidate, so a pair whose other query was
// settled by the filter (most of them when the entries are few) cost a full second column step; here a lane's
// chain is half as long, and a workgroup's 256 lanes still hold every pair of the item (no refill).
template <int W, bool CMP, class Fetch>
__device__ __forceinline__ void bv_dp_mono(const EdBvArgs &A, const uint32_t *peq, uint32_t ns, uint32_t q1,
                                           uint32_t q2, uint32_t n1, uint32_t n2, Fetch fetch, uint32_t &c_dp_pairs,
                                           uint32_t &c_in_band, uint32_t &c_blocks, uint32_t &c_dp_cand,
                                           uint32_t &c_live) {
    using SH = BvShape<W>;
    const uint32_t lane = threadIdx.x & 63, e = threadIdx.x >> 1, sq = threadIdx.x & 1;
    const uint32_t w = A.w, w1 = A.w + 1;
    const uint16_t *rmap = (const uint16_t *)(peq + A.rmap_dw);
    uint32_t j = 0;
    bool run = false;
    if (e < ns) {
        bool a1, a2;
        fetch(e, j, a1, a2);
        run = sq ? a2 : a1;
        if (sq == 0) c_dp_cand += 1;  // an entry counts once
    }
    bool active = run;
    c_dp_pairs += (uint32_t)run;
    const uint32_t m = active ? A.len[j] : 0u, n = sq ? n2 : n1;
    const uint16_t *stream = active ? A.bsym + A.soff[j] : A.bsym;  // idle lanes read a valid stream
    uint32_t r = w1;
    BvState<SH::KF> S;
    bv_init<W>(S);
    uint32_t cur[16], nxt[16];
    bv_load_block(cur, stream, 0);
    for (uint32_t kb = 0; __any(active); ++kb) {
        c_blocks += (uint32_t)active;
        c_live += (uint32_t)(active && run);
        bv_load_block(nxt, stream, kb + 1);  // streams carry one spare block
        const uint32_t j0 = 32 * kb, base = (kb + 1) * 8 + 4 * sq;
        const bool here = active && run && m > j0 && m <= j0 + 32;
#if NMZ_ED_PF > 0
        if constexpr (!CMP || NMZ_ED_PF_CMP) {
            if (__any(here)) {
                bv_block1_pf<W, CMP, true>(S, peq, rmap, cur, base, j0, m, n, run, r, w1);
            } else {
                bv_block1_pf<W, CMP, false>(S, peq, rmap, cur, base, j0, m, n, run, r, w1);
            }
        } else
#endif
        {
            if (__any(here)) {
                bv_block1<W, CMP, true>(S, peq, rmap, cur, base, j0, m, n, run, r, w1);
            } else {
                bv_block1<W, CMP, false>(S, peq, rmap, cur, base, j0, m, n, run, r, w1);
            }
        }
        S.T += 32 - __builtin_popcount(S.acc);
        if (run && bv_lower_bound<W>(S, S.T) > w) run = false;
#pragma unroll
        for (int k = 0; k < 16; ++k) cur[k] = nxt[k];
        const bool fin = active && !run;
        if (__any(fin))
            bv_publish(A, fin, j, q1, q2, sq == 1, sq ? w1 : r, sq ? r : w1, lane, w, c_in_band);
        if (fin) active = false;
    }
}

template <int W, bool CMP>
__global__ __launch_bounds__(256) NMZ_ED_BV_ATTR void k_ed_bv(EdBvArgs A) {
    extern __shared__ uint32_t peq[];
    // pool counter lives after the Peq tables (a static __shared__ variable
    // would shift the dynamic region off 8-byte alignment: misaligned ds_read_b64)
    uint32_t &pool_next = peq[A.lds_dw];
    const uint32_t nblk = gridDim.x, per_xcd = nblk / 8;
    const uint32_t lb = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    const uint32_t wpc = A.rq / 2;  // workgroups per chunk
    const uint64_t lchunk = lb / wpc;
    if (lchunk >= A.n_chunks) return;
    // the lchunk-th chunk of the plan: row b (binary search of the per-row chunk starts), chunk cr of the row
    uint32_t lo = 0, hi = A.G;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (A.chunk_start[mid] <= lchunk) lo = mid; else hi = mid;
    }
    const uint32_t b = lo;
    const uint32_t cr = (uint32_t)(lchunk - A.chunk_start[b]);
    const uint32_t q1 = A.rq * b + 2 * (lb % wpc), q2 = q1 + 1;
    if (q1 >= A.N) return;  // whole workgroup
    // the shard owns whole 64-query blocks (ed_block_shard, as in the two-phase search); q1 is even, so q1 and q2
    // share one block
    if (ed_block_shard(q1 / 64, A.n_shards) != A.shard) return;
    const bool has2 = q2 < A.N;
    const uint32_t n1 = A.len[q1], n2 = has2 ? A.len[q2] : 0;
    const uint32_t c0 = A.rq * b + A.pool * cr;
    const uint32_t c1 = min(c0 + A.pool, A.N);
    const uint32_t pool_lo = max(c0, q1 + 1);
    const uint32_t pool_n = c1 > pool_lo ? c1 - pool_lo : 0;

    // after the pool counter and the survivor count (16-byte aligned: lds_dw is a multiple of 4): the two queries'
    // q-gram profiles, then the pool's survivors (u16: pool index | run1 << 14 | run2 << 15)
    uint32_t &n_surv = peq[A.lds_dw + 1];
    uint32_t *qprof = peq + A.lds_dw + 4;
    uint16_t *surv = (uint16_t *)(qprof + 2 * ED_QG_DW);
    if (threadIdx.x == 0) {
        pool_next = 256;
        n_surv = 0;
    }
    if (A.prof && threadIdx.x < 2 * ED_QG_DW) {
        const uint32_t q = threadIdx.x < ED_QG_DW ? q1 : q2, w = threadIdx.x % ED_QG_DW;
        qprof[threadIdx.x] = (q < A.N) ? ((const uint32_t *)A.prof)[(uint64_t)q * ED_QG_DW + w] : 0u;
    }
    __syncthreads();
    // work counters (A.counters): DP pairs, in-band pairs, lane blocks, DP candidates, live query-blocks, q-gram
    uint32_t c_dp_pairs = 0, c_in_band = 0, c_blocks = 0, c_dp_cand = 0, c_live = 0, c_qgram = 0;
    // ---- the pool's pairs that need a DP, decided for all candidates at once (all 256 threads) ----
    // Out of the length band (|n - m| > w) or settled by the q-gram bound (L1 > 4w): w + 1, nothing to list
    // (k_knn_fill). An empty trace within the length band: n + m <= w, listed here. The DP loop below then
    // draws only survivors, so lanes never stall the wave on candidates that need no DP, and a workgroup whose
    // pool has no survivor builds no Peq tables at all. Four candidates per thread per step keep their loads
    // in flight together.
    for (uint32_t c4 = 4 * threadIdx.x; c4 < pool_n; c4 += 4 * 256) {
        uint32_t mm[4], l1[4], l2[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) mm[u] = c4 + u < pool_n ? A.len[pool_lo + c4 + u] : 0u;
        if (A.prof) {
#pragma unroll
            for (int u = 0; u < 4; ++u)
                qg_l1x2(A.prof + (uint64_t)(pool_lo + min(c4 + u, pool_n - 1)) * (ED_QG_DW / 4), (const uint4 *)qprof,
                        (const uint4 *)(qprof + ED_QG_DW), l1[u], l2[u]);
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const uint32_t c = c4 + u;
            if (c >= pool_n) break;
            const uint32_t jj = pool_lo + c;
            const bool vv2 = has2 && jj > q2;
            const int32_t dd1 = (int32_t)mm[u] - (int32_t)n1, dd2 = (int32_t)mm[u] - (int32_t)n2;
            const int32_t w = (int32_t)A.w;
            bool a1 = dd1 <= w && dd1 >= -w, a2 = vv2 && dd2 <= w && dd2 >= -w;
            if (a1 && (n1 == 0 || mm[u] == 0)) {
                const uint64_t r = n1 + mm[u];
                bv_knn_insert(A.knn + (uint64_t)jj * A.k, A.k, (r << 32) | q1);
                bv_knn_insert(A.knn + (uint64_t)q1 * A.k, A.k, (r << 32) | jj);
                c_in_band += 1;
                a1 = false;
            }
            if (a2 && (n2 == 0 || mm[u] == 0)) {
                const uint64_t r = n2 + mm[u];
                bv_knn_insert(A.knn + (uint64_t)jj * A.k, A.k, (r << 32) | q2);
                bv_knn_insert(A.knn + (uint64_t)q2 * A.k, A.k, (r << 32) | jj);
                c_in_band += 1;
                a2 = false;
            }
            if (A.prof) {  // q-gram bound: L1 > 4w => ED_w = w + 1, no DP
                const bool f1 = a1 && l1[u] > 4 * A.w, f2 = a2 && l2[u] > 4 * A.w;
                c_qgram += (uint32_t)f1 + (uint32_t)f2;
                a1 = a1 && !f1;
                a2 = a2 && !f2;
            }
            if (a1 || a2) surv[atomicAdd(&n_surv, 1u)] = (uint16_t)(c | ((uint32_t)a1 << 14) | ((uint32_t)a2 << 15));
        }
    }
    __syncthreads();
    const uint32_t ns = n_surv;
    if (ns > 0) {  // the two queries' Peq tables (uniform branch: ns is read after the barrier)
        uint4 *p4 = (uint4 *)peq;
        for (uint32_t i = threadIdx.x; i < A.lds_dw / 4; i += 256) p4[i] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x == 0) peq[A.lds_dw + 3] = 0;  // compact tables: rows claimed
        __syncthreads();
        bv_peq_build<W, CMP>(peq, A.rmap_dw, A.claim_dw, A.row_bytes, &peq[A.lds_dw + 3], A.bsym + A.soff[q1], n1,
                             has2 ? A.bsym + A.soff[q2] : nullptr, n2);
        __syncthreads();
    }

    bv_dp_run<W, CMP>(A, peq, pool_next, ns, q1, q2, n1, n2, has2,
                 [&](uint32_t i, uint32_t &jj, bool &a1, bool &a2) {
                     const uint32_t e = surv[i];
                     jj = pool_lo + (e & 0x3fffu);
                     a1 = (e >> 14) & 1u;
                     a2 = e >> 15;
                 },
                 c_dp_pairs, c_in_band, c_blocks, c_dp_cand, c_live);
    bv_flush_counters(A.counters, c_dp_pairs, c_in_band, c_blocks, c_dp_cand, c_live, c_qgram);
}

// ---------------------------------------------------------------------------
// Two-phase search (nmz_internal.h EdQgArgs): filter tiles, then DP work items.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t qg_l1_reg(const uint4 (&c)[ED_QG_DW / 4], const uint4 *q) {
    uint32_t s = 0;
#pragma unroll
    for (int r = 0; r < (int)ED_QG_DW / 4; ++r) {
        const uint4 a = q[r];
        s = __builtin_amdgcn_sad_u8(c[r].x, a.x, s);
        s = __builtin_amdgcn_sad_u8(c[r].y, a.y, s);
        s = __builtin_amdgcn_sad_u8(c[r].z, a.z, s);
        s = __builtin_amdgcn_sad_u8(c[r].w, a.w, s);
    }
    return s;
}

// One tile: queries [64 qb, 64 qb + 64) x candidates [256 cb, 256 cb + 256), pairs j > q only (the shard's tile
// list: csrc/ed.hip ed_bv_two_phase).
// the tile of hardware block b: XCD b % 8 takes a contiguous eighth of the list (its superblocks' profiles stay in
// that XCD's L2); the grid is a multiple of 8
__device__ __forceinline__ uint64_t qg_tile_of_block() {
    const uint64_t per = gridDim.x / 8;
    return (uint64_t)(blockIdx.x % 8) * per + blockIdx.x / 8;
}

template <bool COUNT>
__global__ __launch_bounds__(256) void k_ed_qg_filter(EdQgArgs A) {
    __shared__ uint4 qp[64][ED_QG_DW / 4];
    __shared__ uint32_t qlen[64];
    const uint64_t t = qg_tile_of_block();
    if (t >= A.n_tiles) return;
    if (!COUNT && A.abort && *A.abort) return;  // the search's sizes differ from the cached ones: write nothing
    const uint64_t tq = A.tiles[t];
    const uint32_t qb = (uint32_t)(tq >> 32), cb = (uint32_t)tq;
    for (uint32_t i = threadIdx.x; i < 64 * (ED_QG_DW / 4); i += 256) {
        const uint32_t q = 64 * qb + i / (ED_QG_DW / 4);
        qp[i / (ED_QG_DW / 4)][i % (ED_QG_DW / 4)] =
            q < A.N ? A.prof[(uint64_t)q * (ED_QG_DW / 4) + i % (ED_QG_DW / 4)] : make_uint4(0, 0, 0, 0);
    }
    if (threadIdx.x < 64) qlen[threadIdx.x] = 64 * qb + threadIdx.x < A.N ? A.len[64 * qb + threadIdx.x] : 0u;
    __syncthreads();
    const uint32_t j = 256 * cb + threadIdx.x, lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const bool jv = j < A.N;
    const uint32_t m = jv ? A.len[j] : 0u;
    uint4 cp[ED_QG_DW / 4];
#pragma unroll
    for (int r = 0; r < (int)ED_QG_DW / 4; ++r)
        cp[r] = jv ? A.prof[(uint64_t)j * (ED_QG_DW / 4) + r] : make_uint4(0, 0, 0, 0);
    // empty traces (n + m <= w results, listed here) are rare: a tile without one runs the loop without that path
    const bool any_empty =
        __syncthreads_or((jv && m == 0) || (threadIdx.x < 64 && 64 * qb + threadIdx.x < A.N && qlen[threadIdx.x] == 0));
    uint32_t c_qgram = 0, c_in_band = 0;
    auto body = [&](uint32_t pp, auto empty_tag) {
        constexpr bool EMPTY = decltype(empty_tag)::value;
        const uint32_t q1 = 64 * qb + 2 * pp, q2 = q1 + 1;
        const uint32_t n1 = qlen[2 * pp], n2 = qlen[2 * pp + 1];
        const int32_t dd1 = (int32_t)m - (int32_t)n1, dd2 = (int32_t)m - (int32_t)n2, W = (int32_t)A.w;
        bool a1 = jv && j > q1 && dd1 <= W && dd1 >= -W;
        bool a2 = jv && q2 < A.N && j > q2 && dd2 <= W && dd2 >= -W;
        if constexpr (EMPTY) {
            if (a1 && (n1 == 0 || m == 0)) {  // an empty trace: n + m <= w, listed once (count pass)
                if (COUNT) {
                    const uint64_t r = n1 + m;
                    bv_knn_insert(A.knn + (uint64_t)j * A.k, A.k, (r << 32) | q1);
                    bv_knn_insert(A.knn + (uint64_t)q1 * A.k, A.k, (r << 32) | j);
                    c_in_band += 1;
                }
                a1 = false;
            }
            if (a2 && (n2 == 0 || m == 0)) {
                if (COUNT) {
                    const uint64_t r = n2 + m;
                    bv_knn_insert(A.knn + (uint64_t)j * A.k, A.k, (r << 32) | q2);
                    bv_knn_insert(A.knn + (uint64_t)q2 * A.k, A.k, (r << 32) | j);
                    c_in_band += 1;
                }
                a2 = false;
            }
        }
        // q-gram bound: L1 > 4w => ED_w = w + 1, no DP
        const bool f1 = a1 && qg_l1_reg(cp, qp[2 * pp]) > 4 * A.w;
        const bool f2 = a2 && qg_l1_reg(cp, qp[2 * pp + 1]) > 4 * A.w;
        c_qgram += (uint32_t)f1 + (uint32_t)f2;
        a1 = a1 && !f1;
        a2 = a2 && !f2;
        const bool sv = a1 || a2;
        const uint64_t mask = __ballot(sv);
        if (COUNT && A.recs && mask) {  // the survivors for the scatter pass: one record per (wave, pair)
            const uint64_t m1 = __ballot(a1), m2 = __ballot(a2);
            if (lane == 0) {
                const uint32_t sp = blockIdx.x % ED_REC_STRIPES;
                const uint32_t r = atomicAdd(A.n_rec + sp * ED_REC_LINE, 1u);
                if (r < A.rec_cap) {
                    const uint64_t slot = (uint64_t)sp * A.rec_cap + r;
                    A.recs[2 * slot] = make_uint4(q1 >> 1, 256 * cb + 64 * wave, (uint32_t)m1, (uint32_t)(m1 >> 32));
                    A.recs[2 * slot + 1] = make_uint4((uint32_t)m2, (uint32_t)(m2 >> 32), 0u, 0u);
                }
            }
        }
        if (mask) {
            const uint32_t leader = (uint32_t)__ffsll((unsigned long long)mask) - 1;
            const uint32_t n = (uint32_t)__popcll(mask), p = q1 >> 1;
            uint32_t base = 0;
            if (lane == leader) base = COUNT ? atomicAdd(&A.cnt[p], n) : A.poff[p] + atomicSub(&A.cnt[p], n) - n;
            if (!COUNT) {
                base = __shfl(base, leader, 64);
                const uint64_t e = (uint64_t)base + __popcll(mask & ((1ull << lane) - 1));
                if (sv && e < A.ent_cap) A.ent[e] = j | ((uint32_t)a1 << 30) | ((uint32_t)a2 << 31);
            }
        }
    };
    const uint32_t np = min(32u, (A.N - 64 * qb + 1) / 2);  // query pairs of this block
    if (any_empty) {
        for (uint32_t pp = 0; pp < np; ++pp) body(pp, std::true_type{});
    } else {
        for (uint32_t pp = 0; pp < np; ++pp) body(pp, std::false_type{});
    }
    if (COUNT) bv_flush_counters(A.counters, 0, c_in_band, 0, 0, 0, c_qgram);
}

// The write pass from the count pass's records (EdQgArgs::recs): a wave per record -- one count atomic and the
// entries; no profile loads, no L1s, and nothing read for the (wave, pair)s without survivors (most of them: the
// dense per-tile ballots this replaces were 2 KiB per tile, 0.6 GB read per launch on configs[2]).
// (records sit in ED_REC_STRIPES regions of rec_cap: record g of the n_rec is in the stripe whose prefix of counts
// holds it)
static_assert(ED_REC_STRIPES == 64, "the scatter's prefix sums take one wave");
__global__ __launch_bounds__(256) void k_ed_qg_scatter(EdQgArgs A, uint32_t n_rec) {
    __shared__ uint32_t pre[ED_REC_STRIPES];
    const uint32_t lane = threadIdx.x & 63;
    if (threadIdx.x < 64) {  // exclusive prefix sums of the stripes' counts (ED_REC_STRIPES == 64: one wave)
        const uint32_t c = A.rec_cnt[lane];
        uint32_t inc = c;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t v = __shfl_up(inc, o, 64);
            if (lane >= (uint32_t)o) inc += v;
        }
        pre[lane] = inc - c;
    }
    __syncthreads();
    if (A.abort && *A.abort) return;  // the search's sizes differ from the cached ones: write nothing
    const uint32_t nw = gridDim.x * 4;
    for (uint32_t g0 = blockIdx.x * 4 + (threadIdx.x >> 6); g0 < n_rec; g0 += nw) {
        uint32_t lo = 0;  // the last stripe whose prefix is <= g0 (empty stripes share their successor's prefix)
#pragma unroll
        for (uint32_t st = ED_REC_STRIPES / 2; st; st >>= 1)
            if (pre[lo + st] <= g0) lo += st;
        const uint64_t r = (uint64_t)lo * A.rec_cap + (g0 - pre[lo]);
        const uint4 h = A.recs[2 * r], g = A.recs[2 * r + 1];
        const uint64_t m1 = ((uint64_t)h.w << 32) | h.z, m2 = ((uint64_t)g.y << 32) | g.x, mask = m1 | m2;
        uint32_t base = 0;
        if (lane == 0) {  // the pair's next free slots, from its end down (the count pass's count returns to 0)
            const uint32_t c = (uint32_t)__popcll(mask);
            base = A.poff[h.x] + atomicSub(&A.cnt[h.x], c) - c;
        }
        base = __shfl(base, 0, 64);
        const uint64_t bit = 1ull << lane, e = (uint64_t)base + __popcll(mask & (bit - 1));
        if ((mask & bit) && e < A.ent_cap)
            A.ent[e] = (h.y + lane) | ((uint32_t)((m1 & bit) != 0) << 30) | ((uint32_t)((m2 & bit) != 0) << 31);
    }
}

int ed_qg_scatter_launch(const EdQgArgs &A, uint32_t n_rec, hipStream_t st) {
    if (n_rec == 0) return NMZ_OK;
    const uint32_t blocks = (n_rec + 3) / 4 < 8192 ? (n_rec + 3) / 4 : 8192;
    hipLaunchKernelGGL(k_ed_qg_scatter, dim3(blocks), dim3(256), 0, st, A, n_rec);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

int ed_qg_filter_launch(const EdQgArgs &A, bool count, hipStream_t st) {
    if (A.n_tiles == 0) return NMZ_OK;
    NMZ_CHECK(A.n_tiles < (1ULL << 31), "too many traces for one launch");
    const dim3 g((unsigned)((A.n_tiles + 7) / 8 * 8)), b(256);
    if (count) hipLaunchKernelGGL(k_ed_qg_filter<true>, g, b, 0, st, A);
    else hipLaunchKernelGGL(k_ed_qg_filter<false>, g, b, 0, st, A);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// One work item: <= `item` entries of query pair p (items dealt in XCD-remapped order, so a pair's items and
// its neighbours' -- near-duplicates share candidates -- run on one XCD).
template <int W, bool CMP>
__global__ __launch_bounds__(256) NMZ_ED_BV_ATTR void k_ed_bv_dp(EdBvArgs A, const uint32_t *__restrict__ ioff,
                                                                const uint32_t *__restrict__ poff,
                                                                const uint32_t *__restrict__ ent, uint32_t n_pairs,
                                                                uint32_t n_items, uint32_t item,
                                                                const uint32_t *__restrict__ abort) {
    extern __shared__ uint32_t peq[];
    uint32_t &pool_next = peq[A.lds_dw];
    const uint32_t nblk = gridDim.x, per_xcd = nblk / 8;
    const uint32_t lb = (blockIdx.x % 8) * per_xcd + blockIdx.x / 8;
    if (lb >= n_items) return;
    if (abort && *abort) return;  // sizes from a cache that this search's totals contradict: no DP over them
    uint32_t lo = 0, hi = n_pairs;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) / 2;
        if (ioff[mid] <= lb) lo = mid; else hi = mid;
    }
    const uint32_t p = lo, ci = lb - ioff[p];
    const uint32_t e0 = poff[p] + ci * item, e1 = min(poff[p + 1], e0 + item), ns = e1 - e0;
    const uint32_t q1 = 2 * p, q2 = q1 + 1;
    const bool has2 = q2 < A.N;
    const uint32_t n1 = A.len[q1], n2 = has2 ? A.len[q2] : 0;
    {
        uint4 *p4 = (uint4 *)peq;
        for (uint32_t i = threadIdx.x; i < A.lds_dw / 4; i += 256) p4[i] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x == 0) {
            pool_next = 256;
            peq[A.lds_dw + 3] = 0;  // compact tables: rows claimed
        }
    }
    __syncthreads();
    bv_peq_build<W, CMP>(peq, A.rmap_dw, A.claim_dw, A.row_bytes, &peq[A.lds_dw + 3], A.bsym + A.soff[q1], n1,
                         has2 ? A.bsym + A.soff[q2] : nullptr, n2);
    __syncthreads();
    uint32_t c_dp_pairs = 0, c_in_band = 0, c_blocks = 0, c_dp_cand = 0, c_live = 0;
    auto fetch = [&](uint32_t i, uint32_t &jj, bool &a1, bool &a2) {
        const uint32_t e = ent[e0 + i];
        jj = e & 0x3fffffffu;
        a1 = (e >> 30) & 1u;
        a2 = e >> 31;
    };
#if NMZ_ED_DP_MONO
    if (ns <= 128)  // workgroup-uniform
        bv_dp_mono<W, CMP>(A, peq, ns, q1, q2, n1, n2, fetch, c_dp_pairs, c_in_band, c_blocks, c_dp_cand, c_live);
    else
#endif
        bv_dp_run<W, CMP>(A, peq, pool_next, ns, q1, q2, n1, n2, has2, fetch, c_dp_pairs, c_in_band, c_blocks,
                          c_dp_cand, c_live);
    bv_flush_counters(A.counters, c_dp_pairs, c_in_band, c_blocks, c_dp_cand, c_live, 0);
}

int ed_bv_dp_launch(const EdBvArgs &A, const uint32_t *ioff, const uint32_t *poff, const uint32_t *ent,
                    uint32_t n_pairs, uint32_t n_items, uint32_t item, uint32_t bw, bool cmp, hipStream_t st,
                    const uint32_t *abort) {
    if (n_items == 0) return NMZ_OK;
    const unsigned blocks = (n_items + 7) / 8 * 8;  // a multiple of 8 for the XCD remap
    const size_t lds = (size_t)A.lds_dw * 4 + 16;
#define NMZ_DP(Wv, C) \
    hipLaunchKernelGGL((k_ed_bv_dp<Wv, C>), dim3(blocks), dim3(256), lds, st, A, ioff, poff, ent, n_pairs, n_items, \
                       item, abort)
    switch (bw * 2 + (cmp ? 1 : 0)) {
        case 16: NMZ_DP(8, false); break;
        case 17: NMZ_DP(8, true); break;
        case 32: NMZ_DP(16, false); break;
        case 33: NMZ_DP(16, true); break;
        case 64: NMZ_DP(32, false); break;
        case 65: NMZ_DP(32, true); break;
        case 128: NMZ_DP(64, false); break;
        case 129: NMZ_DP(64, true); break;
        default: return fail(NMZ_EINVAL, "internal: band has no bit-parallel kernel");
    }
#undef NMZ_DP
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// ---------------------------------------------------------------------------
// k_ed_bv_query: one or two external query traces against every stored trace of a bit-parallel plan
// (SearchSimilar on a resident store). The queries' Peq rows are built in LDS in the plan's layout
// ([symbol][dword][query], row stride ndw * 8 bytes), so the stored traces' streams of Peq-row byte
// offsets index them unchanged; query symbols the store has never seen carry 0xffff and set no bit (they
// match no stored symbol). Each workgroup takes a pool of stored traces; lanes refill as in k_ed_bv.
// Results go to the queries' k-NN lists only (keys dist << 32 | stored id).
// ---------------------------------------------------------------------------
template <int W, bool CMP>
__global__ __launch_bounds__(256) void k_ed_bv_query(EdBvQueryArgs A) {
    using SH = BvShape<W>;
    extern __shared__ uint32_t peq[];
    uint32_t &pool_next = peq[A.lds_dw];
    const uint32_t pool_lo = blockIdx.x * A.pool;
    const uint32_t pool_n = min(A.pool, A.N - pool_lo);
    const uint32_t n1 = A.nq[0], n2 = A.nq[1];
    const bool has2 = A.n_queries > 1;
    // query q-gram profiles (packed, after the pool counter) and their bucket counts (scratch)
    uint32_t *qprof = peq + A.lds_dw + 4, *qhist = qprof + 2 * ED_QG_DW;
    {
        uint4 *p4 = (uint4 *)peq;
        for (uint32_t i = threadIdx.x; i < A.lds_dw / 4; i += 256) p4[i] = make_uint4(0, 0, 0, 0);
        if (threadIdx.x == 0) {
            pool_next = 256;
            peq[A.lds_dw + 3] = 0;  // compact tables: rows claimed
        }
        for (uint32_t i = threadIdx.x; i < 2 * ED_QG_BUCKETS; i += 256) qhist[i] = 0;
    }
    __syncthreads();
    for (uint32_t q = 0; q < A.n_queries; ++q) {
        const uint16_t *a = A.qs + A.qoff[q];
        for (uint32_t i = threadIdx.x; i + 1 < A.nq[q]; i += 256)
            atomicAdd(&qhist[q * ED_QG_BUCKETS + qg_bucket(a[i], a[i + 1])], 1u);
    }
    bv_peq_build<W, CMP>(peq, A.rmap_dw, A.claim_dw, A.row_bytes, &peq[A.lds_dw + 3], A.qs + A.qoff[0], A.nq[0],
                         A.n_queries > 1 ? A.qs + A.qoff[1] : nullptr, A.n_queries > 1 ? A.nq[1] : 0);
    __syncthreads();
    if (threadIdx.x < 2 * ED_QG_DW) {
        uint32_t w = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) w |= min(qhist[4 * threadIdx.x + b], 255u) << (8 * b);
        qprof[threadIdx.x] = w;
    }
    __syncthreads();
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t w = A.w, w1 = A.w + 1;
    const uint16_t *rmap = (const uint16_t *)(peq + A.rmap_dw);
    uint32_t j = 0, m = 0, r1 = w1, r2 = w1, kb0 = 0;
    bool run1 = false, run2 = false, active = false;
    const uint16_t *stream = A.bsym;
    BvState<SH::KF> S1, S2;
    uint32_t cur[16], nxt[16];
    uint32_t idx = threadIdx.x;
    uint32_t kb = 0;
    bool need = true, first = true;
    auto publish = [&](bool fin) {  // in-band results only (k_knn_fill completes the lists, as in k_ed_bv)
        const bool b1 = fin && r1 <= w, b2 = fin && has2 && r2 <= w;
        if (__any(b1)) bv_knn_insert_wave(A.knn, A.k, b1 ? (((uint64_t)r1 << 32) | j) : UINT64_MAX, lane);
        if (__any(b2)) bv_knn_insert_wave(A.knn + A.k, A.k, b2 ? (((uint64_t)r2 << 32) | j) : UINT64_MAX, lane);
    };
    while (true) {
        while (true) {
            const uint64_t want = __ballot(need);
            if (want == 0) break;
            if (!first) {
                const uint32_t cnt = __popcll(want);
                uint32_t base_idx = 0;
                if (lane == (uint32_t)(__ffsll((unsigned long long)want) - 1)) base_idx = atomicAdd(&pool_next, cnt);
                base_idx = __shfl(base_idx, __ffsll((unsigned long long)want) - 1, 64);
                if (need) idx = base_idx + __popcll(want & ((1ull << lane) - 1));
            }
            first = false;
            if (need) {
                if (idx >= pool_n) {
                    need = false;
                    active = false;
                    stream = A.bsym;
                    bv_load_block(cur, stream, 0);
                } else {
                    j = pool_lo + idx;
                    m = A.len[j];
                    stream = A.bsym + A.soff[j];
                    r1 = w1;
                    r2 = w1;
                    const int32_t dd1 = (int32_t)m - (int32_t)n1, dd2 = (int32_t)m - (int32_t)n2, ww = (int32_t)w;
                    run1 = dd1 <= ww && dd1 >= -ww;
                    run2 = has2 && dd2 <= ww && dd2 >= -ww;
                    if (run1 && (n1 == 0 || m == 0)) { r1 = n1 + m; run1 = false; }
                    if (run2 && (n2 == 0 || m == 0)) { r2 = n2 + m; run2 = false; }
                    if (A.prof && (run1 || run2)) {  // q-gram bound, as in k_ed_bv
                        uint32_t l1, l2;
                        qg_l1x2(A.prof + (uint64_t)j * (ED_QG_DW / 4), (const uint4 *)qprof,
                                (const uint4 *)(qprof + ED_QG_DW), l1, l2);
                        run1 = run1 && l1 <= 4 * w;
                        run2 = run2 && l2 <= 4 * w;
                    }
                    if (run1 || run2) {
                        need = false;
                        active = true;
                        kb0 = kb;
                        bv_init<W>(S1);
                        bv_init<W>(S2);
                        bv_load_block(cur, stream, 0);
                    }
                }
            }
            const bool fin = need && !active && idx < pool_n;
            if (__any(fin)) publish(fin);
        }
        if (!__any(active)) break;
        const uint32_t lkb = active ? kb - kb0 : 0;
        bv_load_block(nxt, stream, lkb + 1);
        const uint32_t j0 = 32 * lkb;
        const uint32_t base = (lkb + 1) * 8;
        const bool here = active && (run1 || run2) && m > j0 && m <= j0 + 32;
#if NMZ_ED_PF2 > 0
        if constexpr (!CMP || NMZ_ED_PF2_CMP) {
            if (__any(here)) {
                bv_block_pf<W, CMP, true>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            } else {
                bv_block_pf<W, CMP, false>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            }
        } else
#endif
        {
            if (__any(here)) {
                bv_block<W, CMP, true>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            } else {
                bv_block<W, CMP, false>(S1, S2, peq, rmap, cur, base, j0, m, n1, n2, run1, run2, r1, r2, w1);
            }
        }
        S1.T += 32 - __builtin_popcount(S1.acc);
        S2.T += 32 - __builtin_popcount(S2.acc);
        if (run1 && bv_lower_bound<W>(S1, S1.T) > w) run1 = false;
        if (run2 && bv_lower_bound<W>(S2, S2.T) > w) run2 = false;
#pragma unroll
        for (int r = 0; r < 16; ++r) cur[r] = nxt[r];
        ++kb;
        const bool fin = active && !run1 && !run2;
        if (__any(fin)) publish(fin);
        if (fin) {
            active = false;
            need = true;
        }
    }
}

int ed_bv_query_launch(const EdBvQueryArgs &A, uint32_t bw, bool cmp, uint32_t blocks, hipStream_t st) {
    const size_t lds = (size_t)A.lds_dw * 4 + 16 + (2 * ED_QG_DW + 2 * ED_QG_BUCKETS) * 4;
    if (lds > 65536) {
        static_assert(ED_BV_LDS_MAX <= 160 * 1024, "LDS");
        NMZ_CHECK(lds <= ED_BV_LDS_MAX, "the query has too many distinct symbols for the bit-parallel search");
#define NMZ_ATTR(Wv, C)                                                                                        \
    if (hipFuncSetAttribute(reinterpret_cast<const void *>(k_ed_bv_query<Wv, C>),                              \
                            hipFuncAttributeMaxDynamicSharedMemorySize, (int)ED_BV_LDS_MAX) != hipSuccess)     \
        return fail(NMZ_EHIP, "hipFuncSetAttribute failed");
        switch (bw * 2 + (cmp ? 1 : 0)) {
            case 16: NMZ_ATTR(8, false) break;
            case 17: NMZ_ATTR(8, true) break;
            case 32: NMZ_ATTR(16, false) break;
            case 33: NMZ_ATTR(16, true) break;
            case 64: NMZ_ATTR(32, false) break;
            case 65: NMZ_ATTR(32, true) break;
            case 128: NMZ_ATTR(64, false) break;
            case 129: NMZ_ATTR(64, true) break;
            default: break;
        }
#undef NMZ_ATTR
    }
#define NMZ_Q(Wv, C) hipLaunchKernelGGL((k_ed_bv_query<Wv, C>), dim3(blocks), dim3(256), lds, st, A)
    switch (bw * 2 + (cmp ? 1 : 0)) {
        case 16: NMZ_Q(8, false); break;
        case 17: NMZ_Q(8, true); break;
        case 32: NMZ_Q(16, false); break;
        case 33: NMZ_Q(16, true); break;
        case 64: NMZ_Q(32, false); break;
        case 65: NMZ_Q(32, true); break;
        case 128: NMZ_Q(64, false); break;
        case 129: NMZ_Q(64, true); break;
        default: return fail(NMZ_EINVAL, "internal: band has no bit-parallel kernel");
    }
#undef NMZ_Q
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// any band w <= 64 runs on the kernels of the smallest template band W >= w
bool ed_bv_supported(uint32_t band) { return band <= 64; }
uint32_t ed_bv_template(uint32_t band) { return band <= 8 ? 8 : band <= 16 ? 16 : band <= 32 ? 32 : 64; }

int ed_bv_launch(const EdBvArgs &A, uint32_t bw, bool cmp, uint64_t blocks, hipStream_t st) {
    // + pool counters, query q-gram profiles, the pool's survivor list (u16, 14-bit pool index)
    if (A.pool > (1u << 14)) return fail(NMZ_EINVAL, "internal: bit-parallel pool above 16384 candidates");
    const size_t lds = (size_t)A.lds_dw * 4 + 16 + 2 * ED_QG_DW * 4 + ((size_t)A.pool * 2 + 15) / 16 * 16;
    NMZ_CHECK(lds <= 65536, "internal: bit-parallel LDS above 64 KiB");
#define NMZ_BV(Wv, C) hipLaunchKernelGGL((k_ed_bv<Wv, C>), dim3((unsigned)blocks), dim3(256), lds, st, A)
    switch (bw * 2 + (cmp ? 1 : 0)) {
        case 16: NMZ_BV(8, false); break;
        case 17: NMZ_BV(8, true); break;
        case 32: NMZ_BV(16, false); break;
        case 33: NMZ_BV(16, true); break;
        case 64: NMZ_BV(32, false); break;
        case 65: NMZ_BV(32, true); break;
        case 128: NMZ_BV(64, false); break;
        case 129: NMZ_BV(64, true); break;
        default: return fail(NMZ_EINVAL, "internal: band has no bit-parallel kernel");
    }
#undef NMZ_BV
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz
