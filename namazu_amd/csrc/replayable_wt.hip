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
#include <cstdlib>
#include <string>
#include <vector>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

constexpr uint32_t WT_BRUTE = 8;       // segments of at most this many events: per-event decisions
constexpr uint32_t WT_NMAX = 4096;     // largest segment the plan kernel sorts in LDS
constexpr uint32_t WT_LDS_MAX = 160 * 1024;
constexpr uint32_t WT_NONE = 0xffffffffu;

struct WtClass {
    uint64_t pn;              // P^len
    uint32_t start, n;        // table segment (C order)
    uint32_t o_lv, o_cm;      // byte offsets in the row image: wavelet levels [K][nw] {bits, ones before};
    uint32_t o_chi, o_e;      //   Cm by rank (+ sentinel); C's high word by position (+ sentinel); e by rank (u16)
    uint32_t o_im, o_ic;      //   bucket indexes (u16): first rank with Cm >= b << msh (257); first position
                              //   with C_hi >= b << 24 (256)
    uint32_t o_pm;            //   per d in [0, n]: {largest rank at positions < d, largest rank at positions >= d}
                              //   (u16 pairs: the maximum of a part none of whose Cm is below its bound)
    uint32_t K, nw;           // levels (2^K > n); words per level (n / 32 + 1)
    uint32_t rS;              // lifting-search rounds (the largest bucket's bit length; set by the plan kernel)
};
static_assert(sizeof(WtClass) == 56, "WtClass layout");

// ---------------------------------------------------------------------------------------------------------------
// plan: one workgroup per (segment, row L). Sorts the segment's keys (Cm << 32 | (0xffff - e) << 16 | position)
// in LDS (bitonic), writes Cm / e by rank and C_hi by position, the two bucket indexes, and the K wavelet levels:
// level l holds bit K-1-l of the ranks, in the order "stably sorted by the top l bits" (the node of the value
// prefix pi starts at pi << (K-l), since the ranks are a permutation of [0, n)), one {32 bits, ones before} pair
// per 32 positions. Also adds the segment's sum of Cm to the row sum (every segment, short ones included).
// ---------------------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_replayable_wt_build(const uint4 *__restrict__ table, uint32_t E,
                                                              WtClass *__restrict__ classes, uint32_t msh, uint32_t mbits,
                                                              uint4 *__restrict__ blob, uint32_t rb16,
                                                              unsigned long long *__restrict__ rowsum) {
    extern __shared__ uint4 wt_build_lds[];
    uint64_t *key = reinterpret_cast<uint64_t *>(wt_build_lds);                 // [WT_NMAX]
    uint32_t *chi = reinterpret_cast<uint32_t *>(key + WT_NMAX);               // [WT_NMAX]
    uint16_t *S0 = reinterpret_cast<uint16_t *>(chi + WT_NMAX);                // [2][WT_NMAX]
    uint32_t *wb = reinterpret_cast<uint32_t *>(S0 + 2 * WT_NMAX);             // [WT_NMAX / 32 + 1]
    uint32_t *cum = wb + WT_NMAX / 32 + 4;                                     // [WT_NMAX / 32 + 1]
    unsigned long long *part = reinterpret_cast<unsigned long long *>(cum + WT_NMAX / 32 + 4);  // [16]
    uint32_t *bmax = reinterpret_cast<uint32_t *>(part + 16);                  // [4]
    uint64_t *tmp = reinterpret_cast<uint64_t *>(bmax + 4);                    // [WT_NMAX] sorted keys
    const uint32_t c = blockIdx.x, L = blockIdx.y, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const WtClass ci = classes[c];
    const uint32_t n = ci.n;
    const uint4 *__restrict__ row = table + (uint64_t)L * E + ci.start;
    char *img = reinterpret_cast<char *>(blob + (uint64_t)L * rb16);
    uint64_t s = 0;
    for (uint32_t i = tid; i < n; i += 1024) s += row[i].z;
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o, 64);
    if (lane == 0) part[wave] = s;
    if (tid < 4) bmax[tid] = 0;
    __syncthreads();
    if (tid == 0) {
        unsigned long long t = 0;
        for (int w = 0; w < 16; ++w) t += part[w];
        atomicAdd(rowsum + L, t);
    }
    if (n <= WT_BRUTE) return;
    uint32_t np = 1, lgp = 0;
    while (np < n) {
        np <<= 1;
        ++lgp;
    }
    for (uint32_t i = tid; i < n; i += 1024) {
        const uint4 q = row[i];
        chi[i] = q.y;
        const uint32_t e = ~q.w;  // < 65536 (the host checks E)
        key[i] = ((uint64_t)q.z << 32) | ((uint64_t)(0xffffu - e) << 16) | i;
    }
    // sort the keys: counting sort on the top lg(np) bits of Cm (uniform in [0, m): ~1 key per bucket), then an
    // insertion sort per bucket (a thread per bucket); a bucket of more than 32 keys (repeated hints: equal Cm)
    // sends the whole segment to a bitonic sort
    {
        uint32_t *bc = reinterpret_cast<uint32_t *>(S0);  // [np] bucket counts, then bucket ends
        const uint32_t sh = mbits > lgp ? mbits - lgp : 0u;
        for (uint32_t b = tid; b < np; b += 1024) bc[b] = 0;
        if (tid == 0) bmax[0] = 0;
        __syncthreads();
        for (uint32_t i = tid; i < n; i += 1024) atomicAdd(&bc[(uint32_t)(key[i] >> 32) >> sh], 1u);
        __syncthreads();
        {  // exclusive scan over np <= 4096 counts: 4 per thread, wave scans, then the 16 wave totals
            const uint32_t b0 = 4 * tid;
            uint32_t c4[4], t = 0;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                c4[k] = b0 + k < np ? bc[b0 + k] : 0u;
                t += c4[k];
                if (c4[k] > 32) atomicMax(bmax, c4[k]);
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
                if (b0 + k < np) bc[b0 + k] = base;  // bucket start (a cursor while scattering, then the end)
                base += c4[k];
            }
        }
        __syncthreads();
        const bool bitonic = bmax[0] > 32;
        if (!bitonic) {
            for (uint32_t i = tid; i < n; i += 1024) {
                const uint64_t kk = key[i];
                tmp[atomicAdd(&bc[(uint32_t)(kk >> 32) >> sh], 1u)] = kk;
            }
            __syncthreads();
            for (uint32_t b = tid; b < np; b += 1024) {  // bucket b: [end of b - 1, end of b)
                const uint32_t lo = b ? bc[b - 1] : 0u, hi = bc[b];
                for (uint32_t i = lo + 1; i < hi; ++i) {
                    const uint64_t v = tmp[i];
                    uint32_t j = i;
                    while (j > lo && tmp[j - 1] > v) {
                        tmp[j] = tmp[j - 1];
                        --j;
                    }
                    tmp[j] = v;
                }
            }
            __syncthreads();
            key = tmp;
        } else {
            for (uint32_t i = n + tid; i < np; i += 1024) key[i] = ~0ull;
            for (uint32_t k = 2; k <= np; k <<= 1)
                for (uint32_t j = k >> 1; j; j >>= 1) {
                    __syncthreads();
                    for (uint32_t i = tid; i < np; i += 1024) {
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
        }
    }
    uint32_t *cm_img = reinterpret_cast<uint32_t *>(img + ci.o_cm);
    uint32_t *chi_img = reinterpret_cast<uint32_t *>(img + ci.o_chi);
    uint16_t *e_img = reinterpret_cast<uint16_t *>(img + ci.o_e);
    for (uint32_t j = tid; j < n; j += 1024) {
        const uint64_t kk = key[j];
        cm_img[j] = (uint32_t)(kk >> 32);
        e_img[j] = (uint16_t)(0xffffu - ((kk >> 16) & 0xffffu));
        S0[kk & 0xffffu] = (uint16_t)j;
        chi_img[j] = chi[j];
    }
    if (tid == 0) {
        cm_img[n] = ~0u;  // sentinels: never below a search bound
        chi_img[n] = ~0u;
    }
    // bucket indexes and their largest bucket (the kernel's lifting searches take bitlen(largest) rounds)
    if (tid < 257) {
        auto lb = [&](uint64_t x) {  // first rank with Cm >= x
            uint32_t lo = 0, hi = n;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if ((key[mid] >> 32) < x) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        const uint32_t a = lb((uint64_t)tid << msh), b = tid < 256 ? lb((uint64_t)(tid + 1) << msh) : n;
        reinterpret_cast<uint16_t *>(img + ci.o_im)[tid] = (uint16_t)a;
        atomicMax(bmax + 2, b - a);
    } else if (tid >= 320 && tid < 320 + 256) {
        const uint32_t bk = tid - 320;
        auto lb = [&](uint64_t x) {  // first position with C_hi >= x
            uint32_t lo = 0, hi = n;
            while (lo < hi) {
                const uint32_t mid = (lo + hi) >> 1;
                if (chi[mid] < x) lo = mid + 1; else hi = mid;
            }
            return lo;
        };
        const uint32_t a = lb((uint64_t)bk << 24), b = lb((uint64_t)(bk + 1) << 24);
        reinterpret_cast<uint16_t *>(img + ci.o_ic)[bk] = (uint16_t)a;
        atomicMax(bmax + 3, b - a);
    }
    __syncthreads();
    if (tid == 0) atomicMax(&classes[c].rS, 32u - __clz(max(bmax[2], bmax[3])));
    // prefix / suffix maxima of the ranks: pm[d] = {max rank at positions < d, max rank at positions >= d};
    // 4 positions per thread, wave scans (up for the prefix, down for the suffix), then the 16 wave totals
    {
        const uint32_t j0 = 4 * tid;
        uint32_t v[4], pre[4], suf[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) v[k] = j0 + k < n ? (uint32_t)S0[j0 + k] : 0u;
        pre[0] = v[0];
        suf[3] = v[3];
#pragma unroll
        for (int k = 1; k < 4; ++k) {
            pre[k] = max(pre[k - 1], v[k]);
            suf[3 - k] = max(suf[4 - k], v[3 - k]);
        }
        uint32_t up = pre[3], dn = suf[0], exu = 0, exd = 0;
        for (int o = 1; o < 64; o <<= 1) {
            const uint32_t a = __shfl_up(up, o, 64), b = __shfl_down(dn, o, 64);
            if (lane >= (uint32_t)o) {
                up = max(up, a);
                exu = max(exu, a);
            }
            if (lane + o < 64) {
                dn = max(dn, b);
                exd = max(exd, b);
            }
        }
        if (lane == 63) wb[wave] = up;
        if (lane == 0) wb[16 + wave] = dn;
        __syncthreads();
        for (uint32_t w = 0; w < 16; ++w) {
            if (w < wave) exu = max(exu, wb[w]);
            if (w > wave) exd = max(exd, wb[16 + w]);
        }
        uint32_t *pm = reinterpret_cast<uint32_t *>(img + ci.o_pm);
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t j = j0 + k;
            if (j <= n) {
                const uint32_t lo = max(exu, k ? pre[k - 1] : 0u);  // positions < j
                const uint32_t hi = j < n ? max(exd, suf[k]) : 0u;  // positions >= j
                pm[j] = lo | hi << 16;
            }
        }
        __syncthreads();  // wb is the level loop's next
    }
    // wavelet levels
    const uint32_t K = ci.K, nw = ci.nw;
    uint2 *lv = reinterpret_cast<uint2 *>(img + ci.o_lv);
    uint16_t *cur = S0, *nxt = S0 + WT_NMAX;
    for (uint32_t l = 0; l < K; ++l) {
        const uint32_t k = K - l, h = 1u << (k - 1);
        for (uint32_t j0 = wave * 64; j0 < nw * 32; j0 += 1024) {
            const uint32_t j = j0 + lane;
            const bool bit = j < n && (cur[j] & h);
            const uint64_t bal = __ballot(bit);
            if (lane == 0) {
                wb[j0 >> 5] = (uint32_t)bal;
                if ((j0 >> 5) + 1 < nw) wb[(j0 >> 5) + 1] = (uint32_t)(bal >> 32);
            }
        }
        __syncthreads();
        if (wave == 0) {  // exclusive scan of the words' popcounts (nw <= 129 words, 3 per lane)
            const uint32_t w0 = 3 * lane;
            const uint32_t c0 = w0 < nw ? __popc(wb[w0]) : 0u, c1 = w0 + 1 < nw ? __popc(wb[w0 + 1]) : 0u,
                           c2 = w0 + 2 < nw ? __popc(wb[w0 + 2]) : 0u;
            const uint32_t t = c0 + c1 + c2;
            uint32_t inc = t;
            for (int o = 1; o < 64; o <<= 1) {
                const uint32_t v = __shfl_up(inc, o, 64);
                if (lane >= (uint32_t)o) inc += v;
            }
            const uint32_t ex = inc - t;
            if (w0 < nw) cum[w0] = ex;
            if (w0 + 1 < nw) cum[w0 + 1] = ex + c0;
            if (w0 + 2 < nw) cum[w0 + 2] = ex + c0 + c1;
        }
        __syncthreads();
        for (uint32_t w = tid; w < nw; w += 1024) lv[l * nw + w] = make_uint2(wb[w], cum[w]);
        for (uint32_t j = tid; j < n; j += 1024) {
            const uint32_t v = cur[j];
            const uint32_t s0 = v & ~(2 * h - 1);  // the node's first position
            const uint32_t r1 = cum[j >> 5] + __popc(wb[j >> 5] & ((1u << (j & 31)) - 1u)) - (s0 >> 1);
            nxt[(v & h) ? s0 + h + r1 : j - r1] = (uint16_t)v;
        }
        __syncthreads();
        uint16_t *t = cur;
        cur = nxt;
        nxt = t;
    }
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

// ones among the first p entries of a level, minus those before the node that starts at s (s >> 1: every node
// before it is whole and half ones)
__device__ __forceinline__ uint32_t wt_ones(const uint2 *__restrict__ lvl, uint32_t s, uint32_t p) {
    const uint2 w = lvl[p >> 5];
    return w.y + __popc(w.x & ((1u << (p & 31)) - 1u)) - (s >> 1);
}

// One seed's statistics over one segment: adds d Hm + (n - d) Hm2 to sum, the segment's wraps to W, and folds its
// maximum key {t, ~e} into key.
template <bool BIG>
__device__ __forceinline__ void wt_seed_class(const WtClass &ci, const char *__restrict__ img,
                                              const uint4 *__restrict__ row, uint64_t h0, uint32_t m, uint64_t mu,
                                              uint32_t m_k64, uint32_t msh, uint64_t &sum, uint32_t &W,
                                              uint64_t &key) {
    const uint32_t n = ci.n;
    const uint64_t H = h0 * ci.pn;
    const uint64_t nH = ~H;
    const uint32_t Hm = BIG ? mod_barrett64(H, m, mu) : mod_barrett_small(H, m, mu);
    const uint32_t t2 = Hm + m_k64;
    const uint32_t Hm2 = BIG ? ((t2 < Hm || t2 >= m) ? t2 - m : t2) : min(t2, t2 - m);
    uint32_t d = 0;
    if (n <= WT_BRUTE) {
        for (uint32_t i = 0; i < n; ++i) wt_decide<BIG>(row[ci.start + i], nH, Hm, Hm2, m, d, W, key);
        sum += (uint64_t)d * Hm + (uint64_t)(n - d) * Hm2;
        return;
    }
    const uint32_t *__restrict__ cm = reinterpret_cast<const uint32_t *>(img + ci.o_cm);
    const uint32_t *__restrict__ chi = reinterpret_cast<const uint32_t *>(img + ci.o_chi);
    const uint16_t *__restrict__ ev = reinterpret_cast<const uint16_t *>(img + ci.o_e);
    const uint16_t *__restrict__ im = reinterpret_cast<const uint16_t *>(img + ci.o_im);
    const uint16_t *__restrict__ ic = reinterpret_cast<const uint16_t *>(img + ci.o_ic);
    const uint32_t *__restrict__ pm = reinterpret_cast<const uint32_t *>(img + ci.o_pm);
    const uint32_t nh = (uint32_t)(nH >> 32);
    const uint32_t XA = m - Hm, XB = m - Hm2;  // t wraps <=> Cm >= X
    // three lifting searches stepped together (every read of a round in flight at once) from the bucket starts:
    // every entry past the bucket is >= the bound, and the sentinel at n ends every probe past the array
    uint32_t pd = ic[nh >> 24], RA = im[XA >> msh], RB = im[XB >> msh];
    for (uint32_t st = (1u << ci.rS) >> 1; st; st >>= 1) {
        const uint32_t a = chi[min(pd + st - 1, n)], b = cm[min(RA + st - 1, n)], c = cm[min(RB + st - 1, n)];
        pd += a < nh ? st : 0u;
        RA += b < XA ? st : 0u;
        RB += c < XB ? st : 0u;
    }
    // d = #{C <= ~H}: #{C_hi < ~H_hi} plus the entries whose high word equals ~H_hi and low word is <= ~H_lo
    // (about n / 2^32 of the queries: the low words come from the table row)
    d = pd;
    if (chi[d] == nh) {
        const uint32_t nl = (uint32_t)nH;
        while (d < n && chi[d] == nh && row[ci.start + d].x <= nl) ++d;
    }
    const uint32_t pmd = pm[d];  // the parts' largest ranks (used when a part has nothing below its bound)
    // descents along R_A's and R_B's paths with the prefix [0, d), branch-free with both reads of a level in
    // flight: counts of ranks >= R, and the deepest level where a part's elements below R branch off (the
    // predecessor's subtree: node start s, prefix offset q)
    const uint2 *__restrict__ lv = reinterpret_cast<const uint2 *>(img + ci.o_lv);
    const uint32_t K = ci.K, nw = ci.nw;
    uint32_t oA = d, oB = d, cA = 0, cB = 0;
    uint32_t lA = WT_NONE, sA = 0, qA = 0, lB = WT_NONE, sB = 0, qB = 0;
    for (uint32_t l = 0; l < K; ++l) {
        const uint32_t h = 1u << (K - l - 1), msk = ~(2 * h - 1);
        const uint2 *__restrict__ lvl = lv + l * nw;
        const uint32_t s1 = RA & msk, p1 = s1 + oA, s2 = RB & msk, p2 = s2 + oB;
        const uint2 w1 = lvl[p1 >> 5], w2 = lvl[p2 >> 5];
        const uint32_t o1 = w1.y + __popc(__builtin_amdgcn_ubfe(w1.x, 0u, p1)) - (s1 >> 1);
        const uint32_t o2 = w2.y + __popc(__builtin_amdgcn_ubfe(w2.x, 0u, p2)) - (s2 >> 1);
        const uint32_t z1 = oA - o1, z2 = oB - o2;
        const bool b1 = RA & h, b2 = RB & h;
        const bool u1 = b1 && z1 != 0;
        const bool u2 = b2 && min(n - s2, h) > z2;  // zeros of the node past the prefix: suffix elements below R_B
        lA = u1 ? l + 1 : lA;
        sA = u1 ? s1 : sA;
        qA = u1 ? z1 : qA;
        lB = u2 ? l + 1 : lB;
        sB = u2 ? s2 : sB;
        qB = u2 ? z2 : qB;
        cA += b1 ? 0u : o1;
        cB += b2 ? 0u : o2;
        oA = b1 ? o1 : z1;
        oB = b2 ? o2 : z2;
    }
    cA += oA;  // the leaf R itself, if in the prefix
    cB += oB;
    W += cA + (n - RB) - cB;
    // predecessor descents: the prefix part takes the largest rank among the first qA entries of node sA, the
    // suffix part the largest among entries qB.. of node sB. A part with nothing below its bound wraps, and its
    // maximum is its largest rank overall (pm). Levels no lane of the wave needs are skipped.
    const bool hasA = d > 0, hasB = d < n, wrapA = lA == WT_NONE, wrapB = lB == WT_NONE;
    if (wrapA || !hasA) lA = K;
    if (wrapB || !hasB) lB = K;
    if (wrapA) sA = pmd & 0xffffu;
    if (wrapB) sB = pmd >> 16;
    const uint32_t l0 = min(lA, lB);
    for (uint32_t l = 0; l < K; ++l) {
        if (!__builtin_amdgcn_ballot_w64(l >= l0)) continue;
        const uint32_t h = 1u << (K - l - 1);
        const uint2 *__restrict__ lvl = lv + l * nw;
        const uint32_t p1 = sA + qA, p2 = sB + qB;
        const uint2 w1 = lvl[p1 >> 5], w2 = lvl[p2 >> 5];
        const uint32_t o1 = w1.y + __popc(__builtin_amdgcn_ubfe(w1.x, 0u, p1)) - (sA >> 1);
        const uint32_t o2 = w2.y + __popc(__builtin_amdgcn_ubfe(w2.x, 0u, p2)) - (sB >> 1);
        const bool a1 = l >= lA, a2 = l >= lB;
        const bool g1 = a1 && o1 != 0;
        const bool g2 = a2 && min(n - sB, 2 * h) > h + o2;  // ones of the node past the prefix
        sA += g1 ? h : 0u;
        qA = g1 ? o1 : qA;
        sB += g2 ? h : 0u;
        qB = a2 ? (g2 ? o2 : qB - o2) : qB;
    }
    if (hasA) {
        const uint32_t t = Hm + cm[sA] - (wrapA ? m : 0u);
        const uint64_t k = ((uint64_t)t << 32) | (0xffffffffu - ev[sA]);
        key = k > key ? k : key;
    }
    if (hasB) {
        const uint32_t t = Hm2 + cm[sB] - (wrapB ? m : 0u);
        const uint64_t k = ((uint64_t)t << 32) | (0xffffffffu - ev[sB]);
        key = k > key ? k : key;
    }
    sum += (uint64_t)d * Hm + (uint64_t)(n - d) * Hm2;
}

// G workgroups per row L: each stages the row image into LDS and takes a contiguous share of the row's 64-seed
// chunks, which its waves take one at a time from an LDS counter.
template <bool BIG>
__global__ __launch_bounds__(1024) void k_replayable_sweep_wt(
    const uint32_t *__restrict__ bucket_off, const uint64_t *__restrict__ sorted_h0,
    const uint32_t *__restrict__ sorted_idx, const uint4 *__restrict__ table, uint32_t E,
    const uint4 *__restrict__ blob, uint32_t rb16, const unsigned long long *__restrict__ rowsum,
    const WtClass *__restrict__ classes, uint32_t n_classes, uint32_t m, uint64_t mu, uint32_t m_k64, uint32_t msh,
    uint32_t G, nmz_sched_stats *__restrict__ stats, unsigned long long *__restrict__ span) {
    extern __shared__ uint4 wt_lds[];
    const uint32_t L = blockIdx.x / G, g = blockIdx.x % G;
    const uint32_t s0 = bucket_off[L], s1 = bucket_off[L + 1];
    const uint32_t nch = (s1 - s0 + 63) / 64;
    const uint32_t c0 = g * nch / G, c1 = (g + 1) * nch / G;
    if (c0 == c1) return;
    if (span && threadIdx.x == 0) atomicMax(span, ~(unsigned long long)wall_clock64());
    uint32_t *ctr = reinterpret_cast<uint32_t *>(wt_lds + rb16);
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
        if (threadIdx.x == 0) *ctr = c0;
    }
    __syncthreads();
    const char *img = reinterpret_cast<const char *>(wt_lds);
    const uint4 *__restrict__ row = table + (uint64_t)L * E;
    const uint64_t rsum = rowsum[L];
    const uint32_t lane = threadIdx.x & 63;
    for (;;) {
        uint32_t ch = 0;
        if (lane == 0) ch = atomicAdd(ctr, 1u);
        ch = __builtin_amdgcn_readfirstlane(ch);
        if (ch >= c1) break;
        const uint32_t j = s0 + ch * 64 + lane;
        const uint64_t h0 = sorted_h0[min(j, s1 - 1)];
        uint64_t sum = 0, key = 0;
        uint32_t W = 0;
        for (uint32_t c = 0; c < n_classes; ++c)
            wt_seed_class<BIG>(classes[c], img, row, h0, m, mu, m_k64, msh, sum, W, key);
        if (j < s1) {
            nmz_sched_stats st;
            st.sum_delay_ns = sum + rsum - (uint64_t)W * m;
            st.max_delay_ns = (int64_t)(key >> 32);
            st.argmax_event = ~(uint32_t)key;
            st.n_fault = 0;
            st.first_fault = NMZ_NONE;
            st.flags = 0;
            stats[sorted_idx[j]] = st;
        }
    }
    if (span) {
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(span + 1, (unsigned long long)wall_clock64());
    }
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
    const char *e = getenv("NMZ_REPLAY_WT");
    return !(e && std::string(e) == "0");
}

// workgroups per row and threads per workgroup (A/B knobs NMZ_WT_G = 1|2|4, NMZ_WT_THREADS = 256..1024)
static uint32_t wt_groups() {
    static const uint32_t g = [] {
        const char *e = getenv("NMZ_WT_G");
        const int v = e ? atoi(e) : 2;
        return (uint32_t)((v == 1 || v == 2 || v == 4 || v == 8) ? v : 2);
    }();
    return g;
}
static uint32_t wt_threads() {
    static const uint32_t t = [] {
        const char *e = getenv("NMZ_WT_THREADS");
        const int v = e ? atoi(e) : 1024;
        return (uint32_t)((v >= 64 && v <= 1024 && v % 64 == 0) ? v : 1024);
    }();
    return t;
}

constexpr size_t WT_BUILD_LDS =
    WT_NMAX * 8 + WT_NMAX * 4 + 2 * WT_NMAX * 2 + 2 * (WT_NMAX / 32 + 4) * 4 + 16 * 8 + 16 + WT_NMAX * 8;

int wt_build(WtState &w, const uint4 *d_table, uint32_t E, const ClassInfo *cls, uint32_t n_cls,
             const ModParams &mod, hipStream_t st) {
    w.on = false;
    if (!wt_enabled() || !mod.m32ok || E == 0 || E > 65536) return NMZ_OK;
    auto r16 = [](uint64_t b) { return (b + 15) & ~15ull; };
    std::vector<WtClass> oc(n_cls);
    uint64_t off = 0;
    for (uint32_t c = 0; c < n_cls; ++c) {
        WtClass &o = oc[c];
        o = WtClass{};
        o.pn = cls[c].pn;
        o.start = cls[c].start;
        o.n = cls[c].count;
        if (o.n >= WT_NMAX) return NMZ_OK;  // keep the order-query sweep (pm and the sort take n < 4,096)
        if (o.n <= WT_BRUTE) continue;
        o.K = bitlen(o.n);  // 2^K > n >= every bound R
        o.nw = o.n / 32 + 1;
        o.o_lv = (uint32_t)off;
        off += r16((uint64_t)o.K * o.nw * 8);
        o.o_cm = (uint32_t)off;
        off += r16((uint64_t)(o.n + 1) * 4);
        o.o_chi = (uint32_t)off;
        off += r16((uint64_t)(o.n + 1) * 4);
        o.o_e = (uint32_t)off;
        off += r16((uint64_t)o.n * 2);
        o.o_im = (uint32_t)off;
        off += r16(257 * 2);
        o.o_ic = (uint32_t)off;
        off += r16(256 * 2);
        o.o_pm = (uint32_t)off;
        off += r16((uint64_t)(o.n + 1) * 4);
    }
    const uint64_t rb = std::max<uint64_t>(16, r16(off));
    if (rb + 16 > WT_LDS_MAX) return NMZ_OK;
    w.rb16 = (uint32_t)(rb / 16);
    w.n_classes = n_cls;
    w.msh = mod.m32 > 255 ? bitlen(mod.m32) - 8 : 0;
    for (const void *f : {reinterpret_cast<const void *>(k_replayable_sweep_wt<false>),
                          reinterpret_cast<const void *>(k_replayable_sweep_wt<true>),
                          reinterpret_cast<const void *>(k_replayable_wt_build)})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)WT_LDS_MAX) != hipSuccess)
            return NMZ_OK;
    const size_t need = Carve::bytes_for(256 * (size_t)w.rb16, 16) + Carve::bytes_for(256, 8) +
                        Carve::bytes_for(n_cls, sizeof(WtClass));
    NMZ_TRY(w.mem.ensure(need));
    Carve cv(w.mem.ptr);
    w.d_blob = cv.take<uint4>(256 * (size_t)w.rb16);
    w.d_rowsum = cv.take<unsigned long long>(256);
    WtClass *d_cls = cv.take<WtClass>(n_cls);
    w.d_classes = d_cls;
    NMZ_HIP(hipMemsetAsync(w.d_rowsum, 0, 256 * 8, st));
    NMZ_HIP(hipMemcpyAsync(d_cls, oc.data(), n_cls * sizeof(WtClass), hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_replayable_wt_build, dim3(n_cls, 256), dim3(1024), WT_BUILD_LDS, st, d_table, E, d_cls,
                       w.msh, bitlen(mod.m32), w.d_blob, w.rb16, w.d_rowsum);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipStreamSynchronize(st));  // the host vector above is pageable
    w.on = true;
    return NMZ_OK;
}

int wt_sweep(const WtState &w, nmz_ctx *ctx, hipStream_t st, const Buckets &b, const uint4 *d_table, uint32_t E,
             const ModParams &mod, nmz_sched_stats *d_stats) {
    const uint32_t G = wt_groups(), nt = wt_threads();
    KernelTimer kt(ctx, st, "replayable_sweep");
    unsigned long long *span = kt.span();
    auto kern = mod.m32 >= 0x80000000u ? k_replayable_sweep_wt<true> : k_replayable_sweep_wt<false>;
    hipLaunchKernelGGL(kern, dim3(256 * G), dim3(nt), w.rb16 * 16u + 16u, st, b.offset, b.sorted_h0, b.sorted_idx,
                       d_table, E, w.d_blob, w.rb16, w.d_rowsum, static_cast<const WtClass *>(w.d_classes),
                       w.n_classes, mod.m32, mod.mu, mod.m_k64, w.msh, G, d_stats, span);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz
