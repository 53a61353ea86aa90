// K1 -- replayable-policy seed sweep (replayablepolicy.go:100-126).
//
//   delay(seed, event) = FNV1a64(seed || hint_e) % uint64(MaxInterval)
//
// Algorithm (MI355X-native, not the reference's per-event hasher):
//  1. Per event, FNV over the hint bytes is an affine map of the incoming
//     state h0 with a correction that depends only on h0's low byte:
//         FNV_hint(h0) = h0 * P^len + C_e[h0 & 0xff]         (mod 2^64)
//     A plan kernel builds C_e[L] for all 256 L (one table row per L).
//  2. Seeds are FNV-hashed once (prefix state h0) and bucketed by h0 & 0xff,
//     so every lane of a wave reads the same table row: table reads are
//     wave-uniform scalar loads.
//  3. Events are grouped by hint length; per (seed, length class) the lane
//     precomputes H = h0*P^len, Hm = H mod m and Hm' = (Hm + 2^64 mod m) mod m:
//         h = H + C (mod 2^64),  carry = C > ~H
//         h mod m = (carry ? Hm' : Hm) + (C mod m)   (one conditional -m)
//  4. Within every (row L, class) segment the table is sorted by C, so the
//     carry is monotone in the position: carry <=> pos >= k(seed), with k
//     found by one binary search per (seed, segment). Per decision the carry
//     is a single compare of a running position counter -- no 64-bit add.
//  5. Per-seed statistics (sum, max with first-index argmax) accumulate in
//     registers; the argmax tie-break uses the key (t << 32 | ~e) so the
//     sorted event order still yields the first original index.
#include <algorithm>
#include <cstring>
#include <cstdlib>
#include <numeric>
#include <string>
#include <vector>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

struct OqClass;

}  // namespace nmz

struct nmz_replayable_plan {
    nmz_ctx *ctx = nullptr;
    uint32_t n_events = 0;
    int64_t max_interval = 0;
    nmz::ModParams mod{};
    uint32_t n_classes = 0;
    nmz::ClassInfo *d_classes = nullptr;
    uint4 *d_table = nullptr;          // [256][E] {C lo, C hi, C mod m, ~e}, C-sorted per class segment
    uint32_t *d_hoff = nullptr;        // hint CSR on the device (dump path)
    uint8_t *d_hbytes = nullptr;
    uint64_t max_seeds = 0;
    nmz::DevBuf seed_scratch;           // h0, buckets, sorted seeds
    nmz::DevBuf partial;                // per-chunk partial (sum, key) per seed
    nmz::DevBuf topk_lists;             // top-k selection scratch (nmz_replayable_sweep_topk_dev)
    nmz::DevBuf plan_mem;
    // order-query statistics (k_replayable_sweep_oq): per-row blobs staged whole into LDS, one blob per pass
    // (a row whose image exceeds LDS is split into passes over disjoint class segments; the per-seed statistics
    // of the passes combine: sums add, maxima max)
    bool oq = false;
    struct OqPass {
        uint32_t c0, c1;                // OqClass range of the pass
        uint64_t off16;                 // first uint4 of the pass's [256][rb16] images in d_oq_blob
        uint32_t rb16;                  // row image bytes / 16
    };
    std::vector<OqPass> oq_passes;
    uint4 *d_oq_blob = nullptr;         // per pass [256][rb16] row images (level arrays {Cm, ~e} + samples of C)
    uint64_t *d_oq_rowsum = nullptr;    // [passes][256] sum of C mod m over the pass's part of the row
    nmz::OqClass *d_oq_classes = nullptr;
    nmz::DevBuf oq_mem;
    nmz::WtState wt;                    // wavelet-tree statistics (k_replayable_sweep_wt, the default when it fits)
    nmz::DevBuf wt_topk;                // their top-k candidates (sums, workgroup maxima, candidates)
    // recorded on the context's stream after the plan's build: a sweep on another stream waits for it on the
    // device (nmz_replayable_plan_create_async returns before the build has run)
    hipEvent_t built = nullptr;
    // the streams the plan's sweeps were enqueued on, each with an event recorded after its latest sweep:
    // destroy waits for exactly that work and the build, not for the whole device or the context's stream
    struct Use {
        hipStream_t st;
        hipEvent_t ev;
    };
    std::vector<Use> uses;
};

namespace nmz {

constexpr uint32_t REPLAY_SEEDS_PER_UNIT_MIN = 64 * 2;

// argmax key mode: f64 bits + v_max_f64 (default) or a u64 compare chain (NMZ_REPLAY_KEY=u64).
// Measured on configs[1]: 0.83 ms vs 0.96 ms per launch. (A strict-greater update on t with a
// tie flag -- 11 full-rate VOP2 per decision, no v_subb / v_max -- measured 0.98 ms.)
static int replay_key_mode() {
    static int k = [] {
        const char *e = ab_env("NMZ_REPLAY_KEY");
        return (e && std::string(e) == "u64") ? 0 : 1;
    }();
    return k;
}

// persistent workgroups (4 waves each) per CU: 8 = 8 waves/SIMD (NMZ_REPLAY_WG for A/B runs)
static uint32_t replay_wg_per_cu() {
    static const uint32_t w = [] {
        const char *e = ab_env("NMZ_REPLAY_WG");
        const int v = e ? atoi(e) : 8;
        return (uint32_t)((v >= 1 && v <= 16) ? v : 8);
    }();
    return w;
}

// seeds per lane (default 2, the fastest measured; NMZ_REPLAY_U=2|4|8 for tuning)
static int replay_u() {
    static int u = [] {
        const char *e = ab_env("NMZ_REPLAY_U");
        int v = e ? atoi(e) : 2;
        return (v == 2 || v == 4 || v == 8) ? v : 2;
    }();
    return u;
}

// ---------------------------------------------------------------------------
// plan: per-(L, event) correction table
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_replayable_table(const uint32_t *__restrict__ hoff,
                                                          const uint8_t *__restrict__ hbytes,
                                                          const uint32_t *__restrict__ perm, uint32_t E,
                                                          uint64_t m, int fast, uint4 *__restrict__ table) {
    const uint32_t pos = blockIdx.x;  // sorted position
    const uint32_t L = threadIdx.x;
    const uint32_t e = perm[pos];
    const uint32_t b0 = hoff[e], b1 = hoff[e + 1];
    uint64_t h = L;
    for (uint32_t i = b0; i < b1; ++i) h = fnv_step(h, hbytes[i]);
    const uint64_t C = h - (uint64_t)L * fnv_pow(b1 - b0);
    const uint32_t cm = fast ? (uint32_t)(C % m) : 0u;
    table[(uint64_t)L * E + pos] = make_uint4((uint32_t)C, (uint32_t)(C >> 32), cm, ~e);
}

// Sort every (row L, class) segment of the table by C (ascending, ties by
// position): rank by counting over the segment through LDS tiles, then
// scatter. O(n_class^2) per row -- ~1e10 compares at E = 4096, well under a ms.
__global__ __launch_bounds__(256) void k_replayable_table_sort(const uint4 *__restrict__ tmp,
                                                               const ClassInfo *__restrict__ classes,
                                                               uint32_t n_classes, uint32_t E,
                                                               uint4 *__restrict__ table) {
    __shared__ uint2 tile[256];
    const uint32_t L = blockIdx.y;
    const uint32_t p0 = blockIdx.x * 256;
    const uint32_t p = p0 + threadIdx.x;
    const uint4 *__restrict__ row = tmp + (uint64_t)L * E;
    uint32_t cs = 0, ce = 0, lo = UINT32_MAX, hi = 0;
    for (uint32_t c = 0; c < n_classes; ++c) {
        const uint32_t a = classes[c].start, b = a + classes[c].count;
        if (p >= a && p < b) cs = a, ce = b;
        // union of the classes this block touches
        if (b > p0 && a < min(E, p0 + 256)) lo = min(lo, a), hi = max(hi, b);
    }
    const uint4 x = p < E ? row[p] : make_uint4(0, 0, 0, 0);
    const uint64_t cx = ((uint64_t)x.y << 32) | x.x;
    uint32_t rank = 0;
    for (uint32_t j0 = lo; j0 < hi; j0 += 256) {
        __syncthreads();
        if (j0 + threadIdx.x < hi) {
            const uint4 y = row[j0 + threadIdx.x];
            tile[threadIdx.x] = make_uint2(y.x, y.y);
        }
        __syncthreads();
        const uint32_t jn = min(256u, hi - j0);
        for (uint32_t jj = 0; jj < jn; ++jj) {
            const uint32_t j = j0 + jj;
            const uint64_t cj = ((uint64_t)tile[jj].y << 32) | tile[jj].x;
            rank += (j >= cs && j < ce && (cj < cx || (cj == cx && j < p))) ? 1u : 0u;
        }
    }
    if (p < E) table[(uint64_t)L * E + cs + rank] = x;
}

// Sort one (class, row L) segment per workgroup in LDS by (C, position) -- the stable C order of
// k_replayable_table_sort -- then gather the table entries in that order. C is an FNV-derived 64-bit value, so a
// counting sort on its top 12 bits leaves ~n/4096 entries per bucket; each bucket is finished by one thread
// (insertion sort). A segment whose largest bucket exceeds SEG_BUCKET_MAX (adversarial C values) takes a bitonic
// sort instead. Segments of up to SEG_SORT_MAX entries; larger classes keep the counting kernel above.
constexpr uint32_t SEG_SORT_MAX = 4096;
constexpr uint32_t SEG_BUCKETS = 4096;
constexpr uint32_t SEG_BUCKET_MAX = 32;

__global__ __launch_bounds__(1024) void k_replayable_table_segsort(const uint4 *__restrict__ tmp,
                                                                   const ClassInfo *__restrict__ classes, uint32_t E,
                                                                   uint4 *__restrict__ table) {
    __shared__ uint64_t key[SEG_SORT_MAX];
    __shared__ uint16_t pos[SEG_SORT_MAX];
    __shared__ uint32_t cnt[SEG_BUCKETS];
    __shared__ uint32_t wsum[16], maxb;
    const ClassInfo ci = classes[blockIdx.x];
    const uint32_t L = blockIdx.y, n = ci.count, t = threadIdx.x;
    if (n > SEG_SORT_MAX || n == 0) return;
    const uint4 *__restrict__ src = tmp + (uint64_t)L * E + ci.start;
    for (uint32_t i = t; i < SEG_BUCKETS; i += blockDim.x) cnt[i] = 0;
    if (t == 0) maxb = 0;
    __syncthreads();
    uint64_t mine[SEG_SORT_MAX / 1024];
#pragma unroll
    for (uint32_t r = 0; r < SEG_SORT_MAX / 1024; ++r) {
        const uint32_t i = r * 1024 + t;
        mine[r] = 0;
        if (i < n) {
            const uint4 q = src[i];
            mine[r] = ((uint64_t)q.y << 32) | q.x;
            atomicAdd(&cnt[mine[r] >> 52], 1u);
        }
    }
    __syncthreads();
    // exclusive scan of the 4096 counts: 4 per thread, wave scans, then the 16 wave totals
    uint32_t c4[4], tot = 0, mx = 0;
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
        c4[r] = cnt[4 * t + r];
        tot += c4[r];
        mx = max(mx, c4[r]);
    }
    const uint32_t lane = t & 63, w = t >> 6;
    uint32_t inc = tot;
    for (uint32_t o = 1; o < 64; o <<= 1) {
        const uint32_t v = __shfl_up(inc, o, 64);
        if (lane >= o) inc += v;
    }
    if (lane == 63) wsum[w] = inc;
    atomicMax(&maxb, mx);
    __syncthreads();
    uint32_t base = inc - tot;
    for (uint32_t j = 0; j < w; ++j) base += wsum[j];
#pragma unroll
    for (uint32_t r = 0; r < 4; ++r) {
        cnt[4 * t + r] = base;  // bucket start, advanced by the scatter below
        base += c4[r];
    }
    __syncthreads();
    if (maxb <= SEG_BUCKET_MAX) {
#pragma unroll
        for (uint32_t r = 0; r < SEG_SORT_MAX / 1024; ++r) {
            const uint32_t i = r * 1024 + t;
            if (i < n) {
                const uint32_t slot = atomicAdd(&cnt[mine[r] >> 52], 1u);
                key[slot] = mine[r];
                pos[slot] = (uint16_t)i;
            }
        }
        __syncthreads();
        // cnt[b] is now the end of bucket b; one thread per bucket sorts its few entries by (C, position)
        for (uint32_t b = t; b < SEG_BUCKETS; b += blockDim.x) {
            const uint32_t e1 = cnt[b], e0 = b ? cnt[b - 1] : 0;
            for (uint32_t i = e0 + 1; i < e1; ++i) {
                const uint64_t k = key[i];
                const uint16_t p = pos[i];
                uint32_t j = i;
                while (j > e0 && (key[j - 1] > k || (key[j - 1] == k && pos[j - 1] > p))) {
                    key[j] = key[j - 1];
                    pos[j] = pos[j - 1];
                    --j;
                }
                key[j] = k;
                pos[j] = p;
            }
        }
        __syncthreads();
    } else {  // bitonic sort of (C, position) padded to a power of two
        uint32_t p2 = 1;
        while (p2 < n) p2 <<= 1;
        for (uint32_t i = t; i < p2; i += blockDim.x) {
            key[i] = i < n ? (((uint64_t)src[i].y << 32) | src[i].x) : UINT64_MAX;
            pos[i] = (uint16_t)i;
        }
        __syncthreads();
        for (uint32_t k = 2; k <= p2; k <<= 1) {
            for (uint32_t j = k >> 1; j > 0; j >>= 1) {
                const uint32_t lj = 31 - __builtin_clz(j);
                for (uint32_t p = t; p < p2 / 2; p += blockDim.x) {
                    const uint32_t i = ((p >> lj) << (lj + 1)) | (p & (j - 1)), l = i + j;
                    const uint64_t ki = key[i], kl = key[l];
                    const uint32_t pi = pos[i], pl = pos[l];
                    const bool gt = ki > kl || (ki == kl && pi > pl);
                    if (((i & k) == 0) == gt) {  // ascending half: swap if i > l; descending half: if i < l
                        key[i] = kl;
                        key[l] = ki;
                        pos[i] = (uint16_t)pl;
                        pos[l] = (uint16_t)pi;
                    }
                }
                __syncthreads();
            }
        }
    }
    uint4 *__restrict__ dst = table + (uint64_t)L * E + ci.start;
    for (uint32_t i = t; i < n; i += blockDim.x) dst[i] = src[pos[i]];
}

// ---------------------------------------------------------------------------
// seed prefix: h0 = FNV(seed bytes)
// ---------------------------------------------------------------------------
// A block's ppt * 256 seeds are contiguous in the CSR: their offsets and (when they fit SEED_LDS_BYTES) their bytes
// are staged in LDS with coalesced loads, and each thread hashes its seeds from LDS. (Per-thread global loads of a
// seed's offsets and bytes made every seed a chain of dependent global loads: ~21 us per 2^20 seeds.)
#ifndef NMZ_SEED_LDS_BYTES
#define NMZ_SEED_LDS_BYTES 16384
#endif
constexpr uint32_t SEED_LDS_BYTES = NMZ_SEED_LDS_BYTES;
constexpr uint32_t SEED_LDS_MAX_SEEDS = NMZ_SEED_LDS_BYTES >= 16384 ? 256 * 16 : 256 * 8;
__global__ __launch_bounds__(256) void k_seed_prefix(const uint32_t *__restrict__ soff,
                                                     const uint8_t *__restrict__ sbytes, uint64_t n,
                                                     uint64_t *__restrict__ h0, uint32_t *__restrict__ rows) {
    // fused bucket histogram (low byte of h0): LDS counts, stored as the block's row of `rows` (Buckets)
    constexpr uint32_t ppt = BUCKET_PT;
    __shared__ uint32_t hist[256];
    __shared__ uint32_t so[SEED_LDS_BYTES ? SEED_LDS_MAX_SEEDS + 1 : 1];
    __shared__ uint32_t sb[SEED_LDS_BYTES ? SEED_LDS_BYTES / 4 : 1];
    hist[threadIdx.x] = 0;
    const uint64_t b0 = (uint64_t)blockIdx.x * 256 * ppt;
    const uint32_t nb = (uint32_t)min<uint64_t>(256 * (uint64_t)ppt, n - b0);
    const bool staged_off = NMZ_SEED_LDS_BYTES > 0 && nb <= SEED_LDS_MAX_SEEDS;
    if (staged_off)
        for (uint32_t i = threadIdx.x; i <= nb; i += 256) so[i] = soff[b0 + i];
    __syncthreads();
    const uint32_t B0 = staged_off ? so[0] : 0u, B1 = staged_off ? so[nb] : 0u;
    // LDS byte off0 + p holds seed byte B0 + p, off0 = the address's offset in its dword, so the whole dwords
    // between the first and last partial dword copy as aligned dwords (no byte outside [B0, B1) is read)
    const uint32_t off0 = (uint32_t)(reinterpret_cast<uintptr_t>(sbytes + B0) & 3u), total = B1 - B0;
    const bool staged = staged_off && off0 + total <= SEED_LDS_BYTES;
    const uint32_t A0 = B0 - off0;  // seed byte positions map to LDS byte (position - A0)
    if (staged) {
        uint8_t *lbw = reinterpret_cast<uint8_t *>(sb);
        const uint32_t head = min((4u - off0) & 3u, total), nint = (total - head) / 4, tail0 = head + 4 * nint;
        if (threadIdx.x < head) lbw[off0 + threadIdx.x] = sbytes[B0 + threadIdx.x];
        const uint32_t *src = reinterpret_cast<const uint32_t *>(sbytes + B0 + head);
        for (uint32_t i = threadIdx.x; i < nint; i += 256) sb[(off0 + head) / 4 + i] = src[i];
        if (threadIdx.x < total - tail0) lbw[off0 + tail0 + threadIdx.x] = sbytes[B0 + tail0 + threadIdx.x];
    }
    __syncthreads();
    const uint8_t *lb = reinterpret_cast<const uint8_t *>(sb);
    for (uint32_t r = 0; r < ppt; ++r) {
        const uint32_t i = r * 256 + threadIdx.x;
        if (i < nb) {
            uint64_t h = FNV_OFFSET;
            if (staged) {
                const uint32_t e = so[i + 1] - A0;
                for (uint32_t t = so[i] - A0; t < e; ++t) h = fnv_step(h, lb[t]);
            } else {
                uint32_t t = soff[b0 + i];
                const uint32_t end = soff[b0 + i + 1];
                // bytes up to a 4-byte boundary, then whole dwords, then the tail
                for (; t < end && (reinterpret_cast<uintptr_t>(sbytes + t) & 3); ++t) h = fnv_step(h, sbytes[t]);
                for (; t + 4 <= end; t += 4) {
                    const uint32_t w = *reinterpret_cast<const uint32_t *>(sbytes + t);
                    h = fnv_step(fnv_step(fnv_step(fnv_step(h, w & 0xff), (w >> 8) & 0xff), (w >> 16) & 0xff), w >> 24);
                }
                for (; t < end; ++t) h = fnv_step(h, sbytes[t]);
            }
            h0[b0 + i] = h;
            atomicAdd(&hist[h & 0xff], 1u);
        }
    }
    __syncthreads();
    rows[(size_t)blockIdx.x * 256 + threadIdx.x] = hist[threadIdx.x];
}

// FNV over the 9 decimal digits of x (< 10^9), most significant first; leading zeros are hashed only once
// `started` (a digit of a more significant part was nonzero)
__device__ __forceinline__ uint64_t fnv_dec9(uint64_t h, uint32_t x, bool &started) {
    constexpr uint32_t P10[9] = {1u, 10u, 100u, 1000u, 10000u, 100000u, 1000000u, 10000000u, 100000000u};
#pragma unroll
    for (int i = 8; i >= 0; --i) {
        const uint32_t d = x / P10[i];  // constant divisor: multiply-high + shift
        x -= d * P10[i];
        started |= d != 0;
        if (started) h = fnv_step(h, '0' + d);
    }
    return h;
}

// FNV(decimal string of v) from state h: strconv.FormatUint(v, 10) bytes
__device__ __forceinline__ uint64_t fnv_decimal_u64(uint64_t h, uint64_t v) {
    const uint64_t e18 = 1000000000000000000ull;
    const uint32_t c2 = (uint32_t)(v / e18);
    const uint64_t r = v - (uint64_t)c2 * e18;
    const uint32_t c1 = (uint32_t)(r / 1000000000ull), c0 = (uint32_t)(r - (uint64_t)c1 * 1000000000ull);
    bool started = false;
    h = fnv_dec9(h, c2, started);
    h = fnv_dec9(h, c1, started);
    h = fnv_dec9(h, c0, started);
    return started ? h : fnv_step(h, '0');
}

// seed prefix of the seeds "seed_lo" .. "seed_lo + n - 1" (decimal strings generated here: no seed CSR), with
// the same fused bucket histogram as k_seed_prefix. decimal(v) = decimal(v / 100) || two digits of v % 100 for
// v >= 100, and a block's 256 ppt consecutive seeds share at most 256 ppt / 100 + 2 prefixes v / 100: one lane per
// prefix hashes it (fnv_decimal_u64, ~300 VALU) into LDS once, then each seed takes its prefix's state and two FNV
// steps (~25 VALU per seed instead of ~300). Seeds below 100, and a block whose range wraps past 2^64, hash
// every seed in full.
constexpr uint32_t DEC_MAX_PREFIX = 64;  // 256 ppt / 100 + 2 <= 64 for ppt = BUCKET_PT <= 16
__global__ __launch_bounds__(256) void k_seed_prefix_decimal(uint64_t seed_lo, uint64_t n, uint64_t *__restrict__ h0,
                                                             uint32_t *__restrict__ rows) {
    constexpr uint32_t ppt = BUCKET_PT;
    __shared__ uint32_t hist[256];
    __shared__ uint64_t ph[DEC_MAX_PREFIX];
    hist[threadIdx.x] = 0;
    const uint64_t b0 = (uint64_t)blockIdx.x * 256 * ppt;
    const uint64_t nb = min<uint64_t>(256 * (uint64_t)ppt, n - b0);  // seeds of this block (>= 1)
    const uint64_t v0 = seed_lo + b0;
    const uint64_t P0 = v0 / 100;
    const uint32_t r0 = (uint32_t)(v0 - P0 * 100);
    const uint32_t np = (r0 + (uint32_t)nb - 1) / 100 + 1;  // prefixes P0 .. P0 + np - 1
    // the shared-prefix form: every seed >= 100, no wrap past 2^64, the prefixes fit the table
    const bool fast = v0 >= 100 && v0 + (nb - 1) >= v0 && np <= DEC_MAX_PREFIX;
    if (fast && threadIdx.x < np) ph[threadIdx.x] = fnv_decimal_u64(FNV_OFFSET, P0 + threadIdx.x);
    __syncthreads();
    for (uint32_t r = 0; r < ppt; ++r) {
        const uint32_t i = r * 256 + threadIdx.x;
        if (i < nb) {
            uint64_t h;
            if (fast) {
                const uint32_t x = r0 + i, q = x / 100, lo = x - q * 100, d1 = lo / 10;
                h = fnv_step(fnv_step(ph[q], '0' + d1), '0' + (lo - d1 * 10));
            } else {
                h = fnv_decimal_u64(FNV_OFFSET, v0 + i);
            }
            h0[b0 + i] = h;
            atomicAdd(&hist[h & 0xff], 1u);
        }
    }
    __syncthreads();
    rows[(size_t)blockIdx.x * 256 + threadIdx.x] = hist[threadIdx.x];
}

// ---------------------------------------------------------------------------
// the sweep (MOD_FAST): persistent waves take work items of up to 64*U seeds
// (U per lane) that share the FNV low byte L, times a chunk of events.
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint32_t vgpr(uint32_t x) {
    // keep a launch constant in a VGPR: VGPR-only VOP2 issues at full rate,
    // the SGPR / literal operand forms at half rate on gfx950
    uint32_t v;
    asm volatile("v_mov_b32 %0, %1" : "=v"(v) : "s"(x));
    return v;
}

__device__ __forceinline__ void vsub(uint32_t &d, uint32_t x) {
    asm("v_sub_u32 %0, %0, %1" : "+v"(d) : "v"(x));
}

// One decision, VOP2 carry/borrow chains only (the forms gfx950 issues at
// ~2.25 cycles; v_cmp_*, v_min/max_u32 and v_addc/v_subb take ~4.1 --
// tools/ubench/valu_patterns.hip, decide_block.hip):
//   vcc = T_t < d                 v_sub_co     (before the seed's carry switch)
//   s   = (vcc ? Hm : Hm2) + Cm   v_cndmask, v_add
//   t   = s < m ? s : s - m       v_sub_co (borrow), v_cndmask
//   key = max(key, t:~e)          v_sub_co / v_subb_co (64-bit borrow), 2 x v_cndmask
//   part += t                     v_add
__device__ __forceinline__ void decide_pos(uint32_t Tt, uint32_t d, uint32_t Hm, uint32_t Hm2, uint32_t Cm,
                                           uint32_t ne, uint32_t mv, uint32_t &klo, uint32_t &khi,
                                           uint32_t &part) {
    uint32_t t0, t1, sv, cv;
    asm("v_sub_co_u32 %[t0], vcc, %[Tt], %[d]\n\t"
        "v_cndmask_b32 %[sv], %[Hm2], %[Hm], vcc\n\t"
        "v_add_u32 %[sv], %[Cm], %[sv]\n\t"
        "v_sub_co_u32 %[cv], vcc, %[sv], %[mv]\n\t"
        "v_cndmask_b32 %[sv], %[cv], %[sv], vcc\n\t"
        "v_sub_co_u32 %[t0], vcc, %[klo], %[ne]\n\t"
        "v_subb_co_u32 %[t1], vcc, %[khi], %[sv], vcc\n\t"
        "v_cndmask_b32 %[klo], %[klo], %[ne], vcc\n\t"
        "v_cndmask_b32 %[khi], %[khi], %[sv], vcc\n\t"
        "v_add_u32 %[part], %[part], %[sv]"
        : [t0] "=&v"(t0), [t1] "=&v"(t1), [sv] "=&v"(sv), [cv] "=&v"(cv), [klo] "+v"(klo), [khi] "+v"(khi),
          [part] "+v"(part)
        : [Tt] "v"(Tt), [d] "v"(d), [Hm] "v"(Hm), [Hm2] "v"(Hm2), [Cm] "v"(Cm), [ne] "v"(ne), [mv] "v"(mv)
        : "vcc");
}

// The same decision with the argmax key kept as the bit pattern of an f64:
// (t << 32 | ~e) with t < 2^30 is a non-negative finite double (bit 63 = 0,
// exponent < 0x7ff; f64 denormals are preserved, the kernel default), whose
// order equals the u64 order, so the 4-instruction u64 compare/select
// becomes one v_max_f64.
__device__ __forceinline__ void decide_f64(uint32_t Tt, uint32_t d, uint32_t Hm, uint32_t Hm2, uint2 q, uint32_t mv,
                                           double &kmax, uint32_t &part) {
    // q = {~e, C mod m}, this seed's own copy from LDS; t replaces C mod m in
    // place, so {~e, t} is already the key's register pair (no v_mov)
    uint32_t t0, tmp, cv;
    uint32_t x = q.y;
    asm("v_sub_co_u32 %[t0], vcc, %[Tt], %[d]\n\t"
        "v_cndmask_b32 %[tmp], %[Hm2], %[Hm], vcc\n\t"
        "v_add_u32 %[x], %[x], %[tmp]\n\t"
        "v_sub_co_u32 %[cv], vcc, %[x], %[mv]\n\t"
        "v_cndmask_b32 %[x], %[cv], %[x], vcc\n\t"
        "v_add_u32 %[part], %[part], %[x]"
        : [t0] "=&v"(t0), [tmp] "=&v"(tmp), [cv] "=&v"(cv), [x] "+v"(x), [part] "+v"(part)
        : [Tt] "v"(Tt), [d] "v"(d), [Hm] "v"(Hm), [Hm2] "v"(Hm2), [mv] "v"(mv)
        : "vcc");
    const double key = __builtin_bit_cast(double, ((uint64_t)x << 32) | q.x);
    asm("v_max_f64 %0, %0, %1" : "+v"(kmax) : "v"(key));
}

// Four decisions of one seed (events T0..T3 of a group) in one asm block: the hazard recognizer
// treats each inline asm conservatively (an s_nop at block boundaries), so one block per four
// decisions instead of one per decision. t overwrites each event's C mod m in place; the four
// keys {~e, t} are folded by key_max4 afterwards, 4+ instructions after their last write
// (0.83 -> 0.80 ms per launch).
__device__ __forceinline__ void decide4(uint32_t T0, uint32_t T1, uint32_t T2, uint32_t T3, uint32_t d, uint32_t Hm,
                                        uint32_t Hm2, uint32_t mv, uint32_t &x0, uint32_t &x1, uint32_t &x2,
                                        uint32_t &x3, uint32_t &part) {
    uint32_t t0, tmp, cv;
#define NMZ_DEC(T, X)                                  \
    "v_sub_co_u32 %[t0], vcc, " T ", %[d]\n\t"         \
    "v_cndmask_b32 %[tmp], %[Hm2], %[Hm], vcc\n\t"     \
    "v_add_u32 " X ", " X ", %[tmp]\n\t"               \
    "v_sub_co_u32 %[cv], vcc, " X ", %[mv]\n\t"        \
    "v_cndmask_b32 " X ", %[cv], " X ", vcc\n\t"       \
    "v_add_u32 %[part], %[part], " X "\n\t"
    asm(NMZ_DEC("%[T0]", "%[x0]") NMZ_DEC("%[T1]", "%[x1]") NMZ_DEC("%[T2]", "%[x2]") NMZ_DEC("%[T3]", "%[x3]")
        : [t0] "=&v"(t0), [tmp] "=&v"(tmp), [cv] "=&v"(cv), [x0] "+v"(x0), [x1] "+v"(x1), [x2] "+v"(x2),
          [x3] "+v"(x3), [part] "+v"(part)
        : [T0] "v"(T0), [T1] "v"(T1), [T2] "v"(T2), [T3] "v"(T3), [d] "v"(d), [Hm] "v"(Hm), [Hm2] "v"(Hm2),
          [mv] "v"(mv)
        : "vcc");
#undef NMZ_DEC
}

__device__ __forceinline__ void key_max4(double &kmax, double a, double b, double c, double d) {
    asm("v_max_f64 %0, %0, %1\n\t"
        "v_max_f64 %0, %0, %2\n\t"
        "v_max_f64 %0, %0, %3\n\t"
        "v_max_f64 %0, %0, %4"
        : "+v"(kmax)
        : "v"(a), "v"(b), "v"(c), "v"(d));
}

// number of entries in the C-sorted range row[lo, lo+n) with C <= x
__device__ __forceinline__ uint32_t count_le(const uint4 *__restrict__ row, uint32_t lo, uint32_t n, uint64_t x) {
    uint32_t k = 0;
    for (uint32_t s = n ? 1u << (31 - __builtin_clz(n)) : 0u; s; s >>= 1) {
        if (k + s <= n) {
            const uint2 c = *reinterpret_cast<const uint2 *>(row + lo + k + s - 1);
            if ((((uint64_t)c.y << 32) | c.x) <= x) k += s;
        }
    }
    return k;
}

// seed r's {~e, C mod m} pair from a 16-B staged read holding seeds 2k, 2k+1
__device__ __forceinline__ uint2 half_of(uint4 v, int hi) { return hi ? make_uint2(v.z, v.w) : make_uint2(v.x, v.y); }

constexpr uint32_t POS_BIAS = 0x40000000u;  // keeps d = BIAS + k - i positive

// Work item = (seed group of <= 64*U seeds sharing the low byte L, chunk of
// `ec` events in the table order). Items are handed out dynamically (one
// global atomic per item) to a persistent grid, so the last round is never a
// half-empty second pass; each item writes its partial (sum, key) per seed
// and k_replayable_merge combines the chunks.
template <int U, int KM>  // KM: 0 = u64 compare chain, 1 = f64 max
__global__ __launch_bounds__(256) void k_replayable_sweep_fast(
    const uint4 *__restrict__ units, const uint32_t *__restrict__ n_units,
    const uint64_t *__restrict__ sorted_h0, const uint4 *__restrict__ table, uint32_t E,
    const ClassInfo *__restrict__ classes, uint32_t n_classes, uint64_t m, uint64_t m_mu, uint32_t m_k64, uint32_t ec,
    uint32_t n_chunks, uint32_t fold_mask, uint32_t *__restrict__ item_counter, uint4 *__restrict__ partial,
    uint64_t part_stride) {
    // per-wave double-buffered staging of 64 table entries in LDS: one
    // coalesced 16-B load per lane fetches the next chunk while the current
    // one is consumed through broadcast LDS reads. An event's slot holds
    // {~e, C mod m} x U: every seed r reads its own pair, and the decision
    // overwrites C mod m with t, leaving the f64 key pair {~e, t} in place.
    static_assert(U % 2 == 0, "staged reads take seeds in pairs");
    constexpr int STR = 2 * U;
    __shared__ __attribute__((aligned(16))) uint32_t stage[4][2][64 * STR];
    const uint32_t wv = threadIdx.x >> 6;
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t m32 = (uint32_t)m;
    const uint32_t mv = vgpr(m32);
    const uint32_t T0 = vgpr(POS_BIAS), T1 = vgpr(POS_BIAS + 1), T2 = vgpr(POS_BIAS + 2), T3 = vgpr(POS_BIAS + 3);
    const uint32_t V4 = vgpr(4u), V1 = vgpr(1u);
    const uint32_t n_items = *n_units * n_chunks;
    uint32_t slot = 0;

    for (;;) {
        uint32_t item = 0;
        if (lane == 0) item = atomicAdd(item_counter, 1u);
        item = __builtin_amdgcn_readfirstlane(__shfl(item, 0, 64));
        if (item >= n_items) break;
        const uint32_t unit = item / n_chunks, chunk = item - unit * n_chunks;
        const uint4 u = units[unit];
        const uint32_t L = __builtin_amdgcn_readfirstlane(u.x);
        const uint32_t start = __builtin_amdgcn_readfirstlane(u.y);
        const uint32_t cnt = __builtin_amdgcn_readfirstlane(u.z);
        const uint32_t e0 = chunk * ec, e1 = min(E, e0 + ec);

        uint64_t h0[U];
        uint32_t sum_lo[U], sum_hi[U], klo[U], khi[U];  // key = max of (t << 32 | ~e); 0 = none
        double kf[U];                                   // the same key as f64 bits (KM 1)
#pragma unroll
        for (int r = 0; r < U; ++r) {
            const uint32_t j = lane + 64 * r;
            h0[r] = (j < cnt) ? sorted_h0[start + j] : 0;
            sum_lo[r] = 0;
            sum_hi[r] = 0;
            klo[r] = 0;
            khi[r] = 0;
            kf[r] = 0.0;
        }
        const uint4 *__restrict__ row = table + (uint64_t)L * E;

        // class containing e0 (few classes: scalar scan)
        uint32_t cc = 0;
        ClassInfo ci = classes[0];
        while (ci.start + ci.count <= e0) ci = classes[++cc];
        uint32_t pos = e0;  // next event (table order) to stage
        uint32_t hi_c = min(e1, ci.start + ci.count);
        uint4 pre = (pos + lane < hi_c) ? row[pos + lane] : make_uint4(0, 0, 0, 0);
        uint32_t Hm[U], Hm2[U], d[U];
        bool fresh = true;
        while (pos < e1) {
            if (fresh) {
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint64_t H = h0[r] * ci.pn;
                    Hm[r] = mod_barrett_small(H, m32, m_mu);
                    const uint32_t t2 = Hm[r] + m_k64;
                    Hm2[r] = min(t2, t2 - m32);
                    // carry(H + C) <=> C > ~H <=> position >= pos + count(C <= ~H)
                    d[r] = POS_BIAS + count_le(row, pos, hi_c - pos, ~H);
                }
                fresh = false;
            }
            const uint32_t n = min(64u, hi_c - pos);
            {
                uint32_t *sw = &stage[wv][slot][lane * STR];
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    sw[2 * r] = pre.w;
                    sw[2 * r + 1] = pre.z;
                }
            }
            // prefetch the next staged chunk (possibly in the next class)
            uint32_t npos = pos + n, nhi = hi_c;
            ClassInfo nci = ci;
            bool nfresh = false;
            if (npos == hi_c && npos < e1) {
                nci = classes[cc + 1];
                nhi = min(e1, nci.start + nci.count);
                nfresh = true;
            }
            // unconditional and clamped to the row: a guarded load became a divergent block whose result
            // the compiler waited for (s_waitcnt vmcnt(0)) right after issuing it. Slots past the chunk's
            // n events are never read, so the clamped lanes' values do not matter.
            pre = row[min(npos + lane, E - 1)];
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
            const uint32_t *__restrict__ sq = stage[wv][slot];
            const uint32_t n4 = n & ~3u;
            // part[r] holds up to 4 << fold_shift delays (< 2^32 since t < m) between folds
            uint32_t part[U];
#pragma unroll
            for (int r = 0; r < U; ++r) part[r] = 0;
            for (uint32_t i = 0, g = 1; i < n4; i += 4, ++g) {
                double kk[U][4];
                // the 4 events' slots as 16-B reads (ds_read_b128: one LDS pass per 4 lane groups,
                // half the LDS cycles of the ds_read2_b64 pairs that 8-B reads compile to)
                uint4 qv[U / 2][4];
                if constexpr (KM == 1) {
#pragma unroll
                    for (int rr = 0; rr < U / 2; ++rr)
#pragma unroll
                        for (int j = 0; j < 4; ++j)
                            qv[rr][j] = *reinterpret_cast<const uint4 *>(sq + (i + j) * STR + 4 * rr);
                }
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint2 *__restrict__ qr = reinterpret_cast<const uint2 *>(sq + i * STR + 2 * r);
                    if constexpr (KM == 1) {
                        const uint2 q0 = half_of(qv[r / 2][0], r & 1), q1 = half_of(qv[r / 2][1], r & 1);
                        const uint2 q2 = half_of(qv[r / 2][2], r & 1), q3 = half_of(qv[r / 2][3], r & 1);
                        uint32_t x0 = q0.y, x1 = q1.y, x2 = q2.y, x3 = q3.y;
                        decide4(T0, T1, T2, T3, d[r], Hm[r], Hm2[r], mv, x0, x1, x2, x3, part[r]);
                        kk[r][0] = __builtin_bit_cast(double, ((uint64_t)x0 << 32) | q0.x);
                        kk[r][1] = __builtin_bit_cast(double, ((uint64_t)x1 << 32) | q1.x);
                        kk[r][2] = __builtin_bit_cast(double, ((uint64_t)x2 << 32) | q2.x);
                        kk[r][3] = __builtin_bit_cast(double, ((uint64_t)x3 << 32) | q3.x);
                    } else {
                        decide_pos(T0, d[r], Hm[r], Hm2[r], qr[0].y, qr[0].x, mv, klo[r], khi[r], part[r]);
                        decide_pos(T1, d[r], Hm[r], Hm2[r], qr[U].y, qr[U].x, mv, klo[r], khi[r], part[r]);
                        decide_pos(T2, d[r], Hm[r], Hm2[r], qr[2 * U].y, qr[2 * U].x, mv, klo[r], khi[r], part[r]);
                        decide_pos(T3, d[r], Hm[r], Hm2[r], qr[3 * U].y, qr[3 * U].x, mv, klo[r], khi[r], part[r]);
                    }
                    vsub(d[r], V4);
                }
                if constexpr (KM == 1) {
#pragma unroll
                    for (int r = 0; r < U; ++r) key_max4(kf[r], kk[r][0], kk[r][1], kk[r][2], kk[r][3]);
                }
                if ((g & fold_mask) == 0) {
#pragma unroll
                    for (int r = 0; r < U; ++r) {
                        const uint32_t lo = sum_lo[r] + part[r];
                        sum_hi[r] += (lo < part[r]);
                        sum_lo[r] = lo;
                        part[r] = 0;
                    }
                }
            }
            for (uint32_t i = n4; i < n; ++i) {  // class / item tail (< 4 events)
#pragma unroll
                for (int r = 0; r < U; ++r) {
                    const uint2 q1 = *reinterpret_cast<const uint2 *>(sq + i * STR + 2 * r);
                    if constexpr (KM == 1)
                        decide_f64(T0, d[r], Hm[r], Hm2[r], q1, mv, kf[r], part[r]);
                    else
                        decide_pos(T0, d[r], Hm[r], Hm2[r], q1.y, q1.x, mv, klo[r], khi[r], part[r]);
                    vsub(d[r], V1);
                }
            }
            // here part holds <= fold_mask groups since the last fold plus the tail
            // (< 4 events): fewer than 4 * (fold_mask + 1) delays, so no overflow
#pragma unroll
            for (int r = 0; r < U; ++r) {
                const uint32_t lo = sum_lo[r] + part[r];
                sum_hi[r] += (lo < part[r]);
                sum_lo[r] = lo;
            }
            slot ^= 1;
            pos = npos;
            if (nfresh) {
                ci = nci;
                ++cc;
                hi_c = nhi;
                fresh = true;
            }
        }
        uint4 *__restrict__ out = partial + (uint64_t)chunk * part_stride + (uint64_t)unit * (64 * U);
#pragma unroll
        for (int r = 0; r < U; ++r) {
            if constexpr (KM == 1) {
                const uint64_t kb = __builtin_bit_cast(uint64_t, kf[r]);
                klo[r] = (uint32_t)kb;
                khi[r] = (uint32_t)(kb >> 32);
            }
            out[lane + 64 * r] = make_uint4(sum_lo[r], sum_hi[r], klo[r], khi[r]);
        }
    }
}

// combine the per-chunk partials of slot g (unit g / 64U, lane-seed g % 64U); false for empty slots
template <int U>
__device__ __forceinline__ bool merge_slot(uint64_t g, const uint4 *__restrict__ units, uint32_t n_units,
                                          const uint32_t *__restrict__ sorted_idx, const uint4 *__restrict__ partial,
                                          uint64_t part_stride, uint32_t n_chunks, nmz_sched_stats &st,
                                          uint32_t &idx) {
    const uint64_t unit = g / (64 * U);
    const uint32_t j = (uint32_t)(g - unit * (64 * U));
    if (unit >= n_units) return false;
    const uint4 u = units[unit];
    if (j >= u.z) return false;
    uint64_t sum = 0, key = 0;
    for (uint32_t c = 0; c < n_chunks; ++c) {
        const uint4 p = partial[(uint64_t)c * part_stride + g];
        sum += ((uint64_t)p.y << 32) | p.x;
        const uint64_t k = ((uint64_t)p.w << 32) | p.z;
        key = k > key ? k : key;
    }
    st.sum_delay_ns = sum;
    st.max_delay_ns = (int64_t)(key >> 32);
    st.argmax_event = ~(uint32_t)key;
    st.n_fault = 0;
    st.first_fault = NMZ_NONE;
    st.flags = 0;
    idx = sorted_idx[u.y + j];
    return true;
}

// combine the per-chunk partials of every seed and scatter to the original index
template <int U>
__global__ __launch_bounds__(256) void k_replayable_merge(const uint4 *__restrict__ units,
                                                          const uint32_t *__restrict__ n_units,
                                                          const uint32_t *__restrict__ sorted_idx,
                                                          const uint4 *__restrict__ partial, uint64_t part_stride,
                                                          uint32_t n_chunks, nmz_sched_stats *__restrict__ stats) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    nmz_sched_stats st;
    uint32_t idx;
    if (merge_slot<U>(g, units, *n_units, sorted_idx, partial, part_stride, n_chunks, st, idx)) stats[idx] = st;
}

// ---------------------------------------------------------------------------
// Order-query statistics (0 < m < 2^32): the per-seed sum, max and first argmax of
// every decision of a (row L, class) segment without deciding event by event.
//
// Inside a segment (C-sorted) every decision is t = (base + Cm) mod m with
// base = Hm on the carry-free prefix [0, d) and Hm2 on [d, n). For a set of
// events with one base b:
//   sum t = |set| b + sum Cm - m #{Cm >= m - b}       (each t wraps at most once)
//   max t = b + max{Cm < m - b}   if that set is non-empty (those t lie in [b, m),
//           b + max Cm - m        otherwise              the wrapped ones in [0, b))
// so a block of events sorted by (Cm, e desc) answers both with one binary
// search for m - b: the count gives the wraps, the entry just below gives the
// maximum and its smallest e. The prefix/suffix split at d is covered by
// aligned blocks of three levels (512, 64, 8 events; each block sorted within
// itself), the 8-event block holding d is decided event by event (which also
// counts d exactly). Per (seed, segment of n events): n/512 + 16 block searches
// instead of n decisions. Segments of <= OQ_BRUTE events are decided event by
// event with wave-uniform table reads. The sum over all segments needs only the
// carry-free counts d and the wrap count W:
//   sum = sum_segments (d Hm + (n - d) Hm2) + sum_row Cm - m W.
//
// LDS image of a row (uint2 units): the three level arrays {Cm, ~e} and the 8-event samples of C, each
// segment's arrays skewed (logical entry i at base + i + i/32) so that the power-of-two strides of a
// binary search land on distinct banks; a block that the segment end cuts short is padded with copies of
// its last (largest) entry, so every search runs over a whole block with immediate-offset reads.
// ---------------------------------------------------------------------------
constexpr uint32_t OQ_S0 = 512, OQ_S1 = 64, OQ_S2 = 8;
constexpr uint32_t OQ_BRUTE = 64;   // segments of at most this many events: per-event decisions
constexpr uint32_t OQ_WG = 1024;    // seeds per workgroup (16 waves share one staged row)
constexpr uint32_t OQ_LDS_MAX = 160 * 1024;

__host__ __device__ constexpr uint32_t oq_skew(uint32_t i) { return i + (i >> 5); }
__host__ __device__ constexpr uint32_t oq_round(uint32_t n, uint32_t s) { return (n + s - 1) / s * s; }

struct OqClass {
    uint64_t pn;            // P^len
    uint32_t start, count;  // table segment (C order)
    uint32_t lv[3];         // level-array bases in the row image (uint2 units)
    uint32_t samp, samp_p2; // sample base; sample slots (a power of two >= ceil(n / 8))
    uint32_t pass;          // the pass (row image) holding this segment
    uint32_t pad[2];
};

// plan: one workgroup per (top block, row L): the top block's entries (C order) sorted by (Cm, ~e) with a
// bitonic network whose runs all end ascending after every stage (the first step of stage k compares an
// element with its mirror in the k-run), so the 8-, 64- and 512-runs are snapshots of the three levels.
// Also writes the 8-event samples of C and adds the block's C mod m to the row sum.
__global__ __launch_bounds__(256) void k_replayable_oq_levels(const uint4 *__restrict__ table, uint32_t E,
                                                              const uint4 *__restrict__ tb_list,
                                                              const OqClass *__restrict__ classes,
                                                              const uint4 *__restrict__ passes,
                                                              uint4 *__restrict__ blob,
                                                              unsigned long long *__restrict__ rowsum) {
    __shared__ uint64_t key[OQ_S0];
    __shared__ unsigned long long part[4];
    const uint4 tb = tb_list[blockIdx.x];  // {class, block start in the segment, size, 0}
    const OqClass ci = classes[tb.x];
    const uint4 ps = passes[ci.pass];      // {image offset lo, hi (uint4 units), rb16, 0}
    const uint32_t L = blockIdx.y, lo = tb.y, size = tb.z, n = ci.count;
    const bool levels = n > OQ_BRUTE;
    const uint4 *__restrict__ row = table + (uint64_t)L * E + ci.start + lo;
    uint2 *img = reinterpret_cast<uint2 *>(blob + ((uint64_t)ps.y << 32 | ps.x) + (uint64_t)L * ps.z);
    rowsum += 256 * ci.pass;
    uint64_t s = 0;
    for (uint32_t i = threadIdx.x; i < OQ_S0; i += 256) {
        if (i < size) {
            const uint4 q = row[i];
            key[i] = ((uint64_t)q.z << 32) | q.w;
            s += q.z;
            if (levels && (i & 7) == 0) img[ci.samp + oq_skew((lo + i) / 8)] = make_uint2(q.x, q.y);
        } else {
            key[i] = UINT64_MAX;
        }
    }
    if (levels && lo == 0)  // sample padding: above every ~H but ~0 (H = 0), where the count is clamped to ns
        for (uint32_t k = (n + 7) / 8 + threadIdx.x; k < ci.samp_p2; k += 256)
            img[ci.samp + oq_skew(k)] = make_uint2(~0u, ~0u);
    for (int o = 32; o; o >>= 1) s += __shfl_xor(s, o, 64);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = s;
    __syncthreads();
    if (threadIdx.x == 0) atomicAdd(rowsum + L, part[0] + part[1] + part[2] + part[3]);
    if (!levels) return;
    const uint32_t p = threadIdx.x;  // one compare-exchange pair per thread
    for (uint32_t k = 2; k <= OQ_S0; k <<= 1) {
        for (uint32_t j = k >> 1; j; j >>= 1) {
            uint32_t i, l;
            if (j == k >> 1) {  // mirror step
                i = (p / j) * k + (p % j);
                l = (p / j) * k + (k - 1 - (p % j));
            } else {
                i = (p / j) * 2 * j + (p % j);
                l = i + j;
            }
            const uint64_t a = key[i], b = key[l];
            if (a > b) {
                key[i] = b;
                key[l] = a;
            }
            __syncthreads();
        }
        const int lv = k == OQ_S2 ? 2 : k == OQ_S1 ? 1 : k == OQ_S0 ? 0 : -1;
        if (lv >= 0) {
            // the level's storage covers the segment rounded up to 512 (level 0) or 64 events
            const uint32_t padlen = oq_round(n, lv == 0 ? OQ_S0 : OQ_S1);
            for (uint32_t i = threadIdx.x; i < OQ_S0 && lo + i < padlen; i += 256) {
                const uint32_t b0 = i & ~(k - 1);
                const uint32_t last = b0 < size ? min(b0 + k, size) - 1 : size - 1;
                const uint64_t q = key[i < size ? i : last];
                const uint2 w = make_uint2((uint32_t)(q >> 32), (uint32_t)q);
                img[ci.lv[lv] + oq_skew(lo + i)] = w;
                // the skew slot after every 32 entries repeats the entry before it, so the entry below phys(idx)
                // is always at phys(idx) - 1
                if (((lo + i) & 31) == 31) img[ci.lv[lv] + oq_skew(lo + i) + 1] = w;
            }
            __syncthreads();
        }
    }
}

// one decision from a table entry {C lo, C hi, Cm, ~e}: counts carry-free events (d) and wraps (W).
// BIG: m >= 2^31, where base + Cm can overflow 32 bits (then the true sum exceeds m, and t = sum - m < m is exact
// modulo 2^32)
template <bool BIG>
__device__ __forceinline__ void oq_decide(uint4 q, uint64_t nH, uint32_t Hm, uint32_t Hm2, uint32_t m, uint32_t &d,
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

// phys offset (from phys(idx)) of element idx + s - 1 in a skewed block, idx a multiple of 2s; and the step
// of phys(idx) when idx grows by s
__host__ __device__ constexpr uint32_t oq_off(uint32_t s) { return s >= 32 ? s - 2 + s / 32 : s - 1; }
__host__ __device__ constexpr uint32_t oq_inc(uint32_t s) { return s >= 32 ? s + s / 32 : s; }

// Interleaved searches over whole sorted blocks (skewed, padded with copies of the block's largest entry):
// chains [0, N0) over 512-blocks, [N0, N0 + N1) over 64-blocks, the rest over 8-blocks, stepped together
// so that every chain ends in the same round (9 dependent rounds of independent LDS reads). Per chain:
// cnt = #{Cm < X} (0..S), cand = the entry just below X, or the block's largest entry when none is below X
// (wrap). pb = phys index of the block's first entry.
template <int N0, int N1, int N2>
__device__ __forceinline__ void oq_search(const uint2 *__restrict__ img, const uint32_t (&pb)[N0 + N1 + N2],
                                          const uint32_t (&X)[N0 + N1 + N2], uint32_t (&cnt)[N0 + N1 + N2],
                                          uint2 (&cand)[N0 + N1 + N2], bool (&wrap)[N0 + N1 + N2]) {
    constexpr int NC = N0 + N1 + N2;
    // byte addresses, so every step is one ds_read_b32 with an immediate offset
    const char *__restrict__ base = reinterpret_cast<const char *>(img);
    uint32_t Q[NC];
#pragma unroll
    for (int k = 0; k < NC; ++k) Q[k] = pb[k] * 8u;
#pragma unroll
    for (uint32_t r = 0; r < 9; ++r) {
#pragma unroll
        for (int k = 0; k < NC; ++k) {
            const uint32_t lg = k < N0 ? 8 : k < N0 + N1 ? 5 : 2;  // log2(S) - 1
            if (r + lg >= 8) {
                const uint32_t st = 1u << (8 - r);
                const uint32_t v = *reinterpret_cast<const uint32_t *>(base + Q[k] + 8u * oq_off(st));
                Q[k] = v < X[k] ? Q[k] + 8u * oq_inc(st) : Q[k];
            }
        }
    }
#pragma unroll
    for (int k = 0; k < NC; ++k) {
        const uint32_t S = k < N0 ? OQ_S0 : k < N0 + N1 ? OQ_S1 : OQ_S2;
        const uint2 first = *reinterpret_cast<const uint2 *>(base + pb[k] * 8u + 8u * oq_skew(S - 1));
        const uint32_t q = (Q[k] >> 3) - pb[k];
        const uint32_t idx = q - ((q * 993u) >> 15);  // phys -> logical (q = idx + idx/32 < 33 * 32)
        const uint2 c = *reinterpret_cast<const uint2 *>(base + Q[k] - 8u);  // idx - 1 (pad slots repeat it)
        const bool all = first.x < X[k];
        cnt[k] = all ? S : idx;
        wrap[k] = !all && idx == 0;
        cand[k] = (all || idx == 0) ? first : c;
        // finish four chains at a time: the compiler would otherwise issue every chain's two final reads
        // at once and spill
        if ((k & 3) == 3) asm volatile("" ::: "memory");
    }
}

// fold one block result into the seed's statistics; side 0 = not this lane's block, 1 = carry-free (Hm),
// 2 = carry (Hm2); rs = the block's real size
__device__ __forceinline__ void oq_accum(int side, uint32_t rs, uint32_t cnt, uint2 cand, bool wrap, uint32_t Hm,
                                         uint32_t Hm2, uint32_t m, uint32_t &W, uint64_t &key) {
    const uint32_t b = side == 2 ? Hm2 : Hm;
    const uint32_t t = b + cand.x - (wrap ? m : 0u);
    const uint64_t k = side ? (((uint64_t)t << 32) | cand.y) : 0ull;
    W += side ? rs - min(cnt, rs) : 0u;
    key = k > key ? k : key;
}

// One seed's statistics over one class segment (replayablepolicy.go:100-114 restated per segment, see above):
// adds d Hm + (n - d) Hm2 to sum, the segment's wraps to W, and folds its maximum key {t, ~e} into key.
// BIG: 2^31 <= m < 2^32 (block results need no change: t = b + Cm - wrap * m is exact modulo 2^32).
template <bool BIG>
__device__ __forceinline__ void oq_seed_class(const OqClass &ci, const uint2 *__restrict__ img,
                                              const uint4 *__restrict__ row, uint64_t h0, uint32_t m, uint64_t mu,
                                              uint32_t m_k64, uint64_t &sum, uint32_t &W, uint64_t &key) {
    const uint32_t n = ci.count, cs = ci.start;
    const uint64_t H = h0 * ci.pn;
    const uint64_t nH = ~H;
    // Hm = H mod m; Hm2 = (Hm + 2^64 mod m) mod m, where for m >= 2^31 the 32-bit add may overflow (then the true
    // value exceeds m and one subtract, modulo 2^32, is exact)
    const uint32_t Hm = BIG ? mod_barrett64(H, m, mu) : mod_barrett_small(H, m, mu);
    const uint32_t t2 = Hm + m_k64;
    const uint32_t Hm2 = BIG ? ((t2 < Hm || t2 >= m) ? t2 - m : t2) : min(t2, t2 - m);
    uint32_t d = 0;
    if (n <= OQ_BRUTE) {
        for (uint32_t i = 0; i < n; ++i) oq_decide<BIG>(row[cs + i], nH, Hm, Hm2, m, d, W, key);
    } else {
        const uint32_t XA = m - Hm, XB = m - Hm2;
        const uint32_t ns = (n + 7) >> 3, nt = (n + OQ_S0 - 1) / OQ_S0;
        // 8-event blocks whose first C is <= ~H are carry-free up to that entry: binary search over the
        // samples (the C of every 8th entry, ascending; slots past ns hold whatever, so the count is clamped)
        uint32_t ks;
        {
            const uint32_t sb = ci.samp;
            uint32_t Q = sb;
            for (uint32_t st = ci.samp_p2 >> 1; st; st >>= 1) {
                const uint2 v = img[Q + oq_off(st)];
                Q = ((((uint64_t)v.y) << 32) | v.x) <= nH ? Q + oq_inc(st) : Q;
            }
            const uint32_t q = Q - sb;
            const uint32_t k0 = q - ((q * 993u) >> 15);
            const uint2 v = img[Q];  // the last slot the lifting cannot reach
            ks = min(k0 + (((((uint64_t)v.y) << 32) | v.x) <= nH ? 1u : 0u), ns);
        }
        const uint32_t b8 = ks ? 8 * (ks - 1) : 0;  // the 8-block holding the carry boundary
        const uint32_t be = b8 + 8;
        {
            const uint32_t nb = min(8u, n - b8);
            // decided event by event; the eight loads are issued together and the updates are selects (a
            // guarded update had let the compiler sink each load into its own branch and wait for it there)
            uint4 q[8];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) q[i] = row[cs + b8 + min(i, nb - 1)];
#pragma unroll
            for (uint32_t i = 0; i < 8; ++i) {
                uint32_t dd = 0, ww = 0;
                uint64_t kk = 0;
                oq_decide<BIG>(q[i], nH, Hm, Hm2, m, dd, ww, kk);
                const bool in = i < nb;
                d += in ? dd : 0u;
                W += in ? ww : 0u;
                key = (in && kk > key) ? kk : key;
            }
        }
        d += b8;
        const uint32_t pad1 = oq_round(n, OQ_S1);
        // level 0: every 512-block of the segment, two at a time (this lane's boundary block is searched
        // and dropped)
        for (uint32_t b = 0; b < nt; b += 2) {
            uint32_t pb[2], X[2], cn[2];
            uint2 cand[2];
            bool wr[2];
            int side[2];
            uint32_t rs[2];
#pragma unroll
            for (int k = 0; k < 2; ++k) {
                const uint32_t lo = min(b + k, nt - 1) * OQ_S0, hi = min(lo + OQ_S0, n);
                side[k] = b + k >= nt ? 0 : hi <= b8 ? 1 : lo >= be ? 2 : 0;
                X[k] = side[k] == 2 ? XB : XA;
                pb[k] = ci.lv[0] + oq_skew(lo);
                rs[k] = hi - lo;
            }
            if (__builtin_amdgcn_ballot_w64(side[0] != 0 || side[1] != 0)) {  // n <= 512: boundary only
                oq_search<2, 0, 0>(img, pb, X, cn, cand, wr);
#pragma unroll
                for (int k = 0; k < 2; ++k) oq_accum(side[k], rs[k], cn[k], cand[k], wr[k], Hm, Hm2, m, W, key);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // level 1: the eight 64-blocks of the boundary 512-block, 4 at a time
            const uint32_t lt = (b8 & ~(OQ_S0 - 1)) + h * 4 * OQ_S1;
            uint32_t pb[4], X[4], cn[4], rs[4];
            int side[4];
            uint2 cand[4];
            bool wr[4], any = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t lo = lt + k * OQ_S1, hi = min(lo + OQ_S1, n);
                side[k] = lo >= n ? 0 : hi <= b8 ? 1 : lo >= be ? 2 : 0;
                any |= side[k] != 0;
                X[k] = side[k] == 2 ? XB : XA;
                pb[k] = ci.lv[1] + oq_skew(min(lo, pad1 - OQ_S1));
                rs[k] = hi - lo;
            }
            if (__builtin_amdgcn_ballot_w64(any)) {
                oq_search<0, 4, 0>(img, pb, X, cn, cand, wr);
#pragma unroll
                for (int k = 0; k < 4; ++k) oq_accum(side[k], rs[k], cn[k], cand[k], wr[k], Hm, Hm2, m, W, key);
            }
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // level 2: the 8-blocks of the boundary 64-block, less the one decided above
            const uint32_t lm = (b8 & ~(OQ_S1 - 1)) + h * 4 * OQ_S2;
            uint32_t pb[4], X[4], cn[4], rs[4];
            int side[4];
            uint2 cand[4];
            bool wr[4], any = false;
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                const uint32_t lo = lm + k * OQ_S2, hi = min(lo + OQ_S2, n);
                side[k] = (lo >= n || lo == b8) ? 0 : lo < b8 ? 1 : 2;
                any |= side[k] != 0;
                X[k] = side[k] == 2 ? XB : XA;
                pb[k] = ci.lv[2] + oq_skew(min(lo, pad1 - OQ_S2));
                rs[k] = hi - lo;
            }
            if (__builtin_amdgcn_ballot_w64(any)) {
                oq_search<0, 0, 4>(img, pb, X, cn, cand, wr);
#pragma unroll
                for (int k = 0; k < 4; ++k) oq_accum(side[k], rs[k], cn[k], cand[k], wr[k], Hm, Hm2, m, W, key);
            }
        }
    }
    sum += (uint64_t)d * Hm + (uint64_t)(n - d) * Hm2;
}

// ACC: a later pass over other class segments of the row -- combine with the statistics of the earlier passes
template <bool ACC>
__device__ __forceinline__ void oq_store(nmz_sched_stats *__restrict__ stats, uint32_t idx, uint64_t sum,
                                         uint64_t key) {
    if constexpr (ACC) {
        const nmz_sched_stats o = stats[idx];
        sum += o.sum_delay_ns;
        const uint64_t ko = ((uint64_t)o.max_delay_ns << 32) | (uint32_t)~o.argmax_event;
        key = ko > key ? ko : key;
    }
    nmz_sched_stats st;
    st.sum_delay_ns = sum;
    st.max_delay_ns = (int64_t)(key >> 32);
    st.argmax_event = ~(uint32_t)key;
    st.n_fault = 0;
    st.first_fault = NMZ_NONE;
    st.flags = 0;
    stats[idx] = st;
}

#ifdef OQ_TRACE
// debug builds only (-DOQ_TRACE): wall_clock64 per (row, wave) at the kernel start [9], after staging [0], at the
// end of each of up to 7 seed chunks [1..7] and after the cooperative tail [8]; read with nmz_debug_oq_trace
__device__ unsigned long long g_oq_trace[256][16][10];
#endif

// One workgroup per row L (256 workgroups, one per CU): the row image is staged into LDS once, then the 16
// waves take the row's seeds in chunks of 64 from an LDS counter. A chunk is a chain of dependent LDS searches
// (~19 us for a wave alone, 20-45 us beside 15 others): with a fixed share of chunks per wave the row waited
// for the waves the SIMD arbiter served last (a row of 4 chunks per wave ended at ~140 us with its median wave
// done at ~110). The row's last partial chunk (ns % 64 seeds) is shared by the waves as they finish: each
// takes a subset of its class segments, and the partial statistics meet in LDS (u64 add and max are
// associative), so it costs about one class chain instead of a whole chunk.
constexpr uint32_t OQ_TAIL = 64;
constexpr uint32_t OQ_TAIL_LDS = OQ_TAIL * 16 + 16;  // {sum, key} per tail seed + the chunk counter

template <bool BIG, bool ACC>
__global__ __launch_bounds__(OQ_WG) void k_replayable_sweep_oq(
    const uint32_t *__restrict__ bucket_off, const uint64_t *__restrict__ sorted_h0,
    const uint32_t *__restrict__ sorted_idx, const uint4 *__restrict__ table, uint32_t E,
    const uint4 *__restrict__ blob, uint32_t rb16, const unsigned long long *__restrict__ rowsum,
    const OqClass *__restrict__ classes, uint32_t n_classes, uint32_t m, uint64_t mu, uint32_t m_k64,
    nmz_sched_stats *__restrict__ stats, unsigned long long *__restrict__ span) {
    extern __shared__ uint4 oq_lds[];
    const uint32_t L = blockIdx.x;
    const uint32_t s0 = bucket_off[L], s1 = bucket_off[L + 1];
    if (s0 == s1) return;
    if (span && threadIdx.x == 0) atomicMax(span, ~(unsigned long long)wall_clock64());
#ifdef OQ_TRACE
    if ((threadIdx.x & 63) == 0) {
        for (int k = 0; k < 10; ++k) g_oq_trace[L][threadIdx.x >> 6][k] = 0;
        g_oq_trace[L][threadIdx.x >> 6][9] = wall_clock64();
    }
#endif
    const uint32_t ns_row = s1 - s0;
    const uint32_t rem = ns_row % 64;
    const uint32_t tail = rem;  // the partial chunk, shared by all waves
    const uint32_t smain = s1 - tail, nch = (smain - s0) / 64;
    unsigned long long *tacc = reinterpret_cast<unsigned long long *>(oq_lds + rb16);  // [OQ_TAIL][2]
    uint32_t *ctr = reinterpret_cast<uint32_t *>(tacc + 2 * OQ_TAIL);
    {
        const uint4 *__restrict__ src = blob + (uint64_t)L * rb16;
        // every load of a pass in flight at once: loads and stores unconditional, indices clamped to the image
        // (guarded loads had compiled to one wait per load plus scratch copies)
        constexpr uint32_t B = 8;  // 128 KB per pass
        for (uint32_t i0 = 0; i0 < rb16; i0 += B * OQ_WG) {
            uint4 v[B];
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) v[k] = src[min(i0 + k * OQ_WG + threadIdx.x, rb16 - 1)];
            // the clamped slots all write the image's last entry to its own place
#pragma unroll
            for (uint32_t k = 0; k < B; ++k) oq_lds[min(i0 + k * OQ_WG + threadIdx.x, rb16 - 1)] = v[k];
        }
        if (tail)
            for (uint32_t i = threadIdx.x; i < 2 * OQ_TAIL; i += OQ_WG) tacc[i] = 0;
        if (threadIdx.x == 0) *ctr = 0;
    }
    __syncthreads();
#ifdef OQ_TRACE
    uint32_t tr_n = 0;
    if ((threadIdx.x & 63) == 0) g_oq_trace[L][threadIdx.x >> 6][tr_n] = wall_clock64();
    ++tr_n;
#endif
    const uint2 *img = reinterpret_cast<const uint2 *>(oq_lds);
    const uint4 *__restrict__ row = table + (uint64_t)L * E;
    const uint64_t rsum = rowsum[L];
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    for (;;) {
        uint32_t ch = 0;
        if (lane == 0) ch = atomicAdd(ctr, 1u);
        ch = __builtin_amdgcn_readfirstlane(ch);
        if (ch >= nch) break;
        const uint32_t j = s0 + ch * 64 + lane;
        const uint64_t h0 = sorted_h0[j];
        uint64_t sum = 0, key = 0;
        uint32_t W = 0;
        for (uint32_t c = 0; c < n_classes; ++c) {
            const OqClass ci = classes[c];
            oq_seed_class<BIG>(ci, img, row, h0, m, mu, m_k64, sum, W, key);
        }
        oq_store<ACC>(stats, sorted_idx[j], sum + rsum - (uint64_t)W * m, key);
#ifdef OQ_TRACE
        if (lane == 0 && tr_n < 8) g_oq_trace[L][wave][tr_n] = wall_clock64();
        ++tr_n;
#endif
    }
    if (tail) {
        // r chunks of <= 64 tail seeds; wave w takes chunk w % r and every P-th class segment from w / r
        const uint32_t r = (tail + 63) >> 6, P = (OQ_WG / 64) / r;
        if (wave < r * P) {
            const uint32_t jj = (wave % r) * 64 + lane, part = wave / r;
            const uint64_t h0 = sorted_h0[smain + min(jj, tail - 1)];
            uint64_t sum = 0, key = 0;
            uint32_t W = 0;
            for (uint32_t c = part; c < n_classes; c += P) {
                const OqClass ci = classes[c];
                oq_seed_class<BIG>(ci, img, row, h0, m, mu, m_k64, sum, W, key);
            }
            if (jj < tail) {
                atomicAdd(tacc + 2 * jj, (unsigned long long)(sum - (uint64_t)W * m));
                atomicMax(tacc + 2 * jj + 1, (unsigned long long)key);
            }
        }
        __syncthreads();
        if (threadIdx.x < tail)
            oq_store<ACC>(stats, sorted_idx[smain + threadIdx.x], tacc[2 * threadIdx.x] + rsum,
                          tacc[2 * threadIdx.x + 1]);
#ifdef OQ_TRACE
        if (lane == 0) g_oq_trace[L][wave][8] = wall_clock64();
#endif
    }
    if (span) {  // one atomic per workgroup: 4,096 same-address atomics at once (one per wave) queue for ~35 us
        __syncthreads();
        if (threadIdx.x == 0) atomicMax(span + 1, (unsigned long long)wall_clock64());
    }
}

// general modulus (m >= 2^30, including uint64(negative duration)): one seed per lane
__global__ __launch_bounds__(256) void k_replayable_sweep_general(
    const uint4 *__restrict__ units, const uint32_t *__restrict__ n_units,
    const uint64_t *__restrict__ sorted_h0, const uint32_t *__restrict__ sorted_idx,
    const uint4 *__restrict__ table, uint32_t E, const ClassInfo *__restrict__ classes,
    uint32_t n_classes, uint64_t m, nmz_sched_stats *__restrict__ stats) {
    const uint32_t wave = __builtin_amdgcn_readfirstlane((blockIdx.x * 256 + threadIdx.x) >> 6);
    const uint32_t lane = threadIdx.x & 63;
    if (wave >= *n_units) return;
    const uint4 u = units[wave];
    const uint32_t L = __builtin_amdgcn_readfirstlane(u.x);
    const uint32_t start = __builtin_amdgcn_readfirstlane(u.y);
    const uint32_t cnt = __builtin_amdgcn_readfirstlane(u.z);
    const uint4 *__restrict__ row = table + (uint64_t)L * E;
    for (uint32_t j = lane; j < cnt; j += 64) {
        const uint64_t h0 = sorted_h0[start + j];
        uint64_t sum = 0;
        int64_t best = INT64_MIN;
        uint32_t arg = NMZ_NONE;
        for (uint32_t c = 0; c < n_classes; ++c) {
            const ClassInfo ci = classes[c];
            const uint64_t H = h0 * ci.pn;
            for (uint32_t i = 0; i < ci.count; ++i) {
                const uint4 qq = row[ci.start + i];
                const uint64_t h = H + (((uint64_t)qq.y << 32) | qq.x);
                const int64_t d = (int64_t)(h % m);
                const uint32_t e = ~qq.w;
                sum += (uint64_t)d;
                if (arg == NMZ_NONE || d > best || (d == best && e < arg)) {
                    best = d;
                    arg = e;
                }
            }
        }
        nmz_sched_stats st;
        st.sum_delay_ns = sum;
        st.max_delay_ns = best;
        st.argmax_event = arg;
        st.n_fault = 0;
        st.first_fault = NMZ_NONE;
        st.flags = 0;
        stats[sorted_idx[start + j]] = st;
    }
}

// maxInterval == 0 (every delay is 0) or no events
__global__ __launch_bounds__(256) void k_stats_constant(uint64_t n, uint32_t E,
                                                        nmz_sched_stats *__restrict__ stats) {
    uint64_t s = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (s >= n) return;
    nmz_sched_stats st;
    stats_empty(st);
    if (E) {
        st.max_delay_ns = 0;
        st.argmax_event = 0;
    }
    stats[s] = st;
}

// full per-decision dump for the first n_dump seeds (parity / debugging path):
// plain FNV over seed bytes || hint bytes, independent of the table
__global__ __launch_bounds__(256) void k_replayable_dump(const uint32_t *__restrict__ soff,
                                                         const uint8_t *__restrict__ sbytes,
                                                         uint64_t n_dump, const uint32_t *__restrict__ hoff,
                                                         const uint8_t *__restrict__ hbytes, uint32_t E,
                                                         uint64_t m, int64_t *__restrict__ out) {
    uint64_t idx = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_dump * E) return;
    const uint64_t s = idx / E;
    const uint32_t e = (uint32_t)(idx % E);
    uint64_t h = FNV_OFFSET;
    for (uint32_t i = soff[s], end = soff[s + 1]; i < end; ++i) h = fnv_step(h, sbytes[i]);
    for (uint32_t i = hoff[e], end = hoff[e + 1]; i < end; ++i) h = fnv_step(h, hbytes[i]);
    out[idx] = m ? (int64_t)(h % m) : 0;
}

constexpr uint32_t REPLAY_EC = 2048;  // events per work item (2048 vs 1024: same sweep time, half the merge reads)

static uint32_t replay_ec() {
    static uint32_t ec = [] {
        const char *e = ab_env("NMZ_REPLAY_EC");
        uint32_t v = e ? (uint32_t)atoi(e) : REPLAY_EC;
        return (v >= 64 && v % 64 == 0) ? v : REPLAY_EC;
    }();
    return ec;
}

// order-query statistics (default) or the per-decision sweep (NMZ_REPLAY_OQ=0, for A/B runs and as the path
// for rows too large for LDS)
static bool replay_oq_enabled() {
    static const bool on = [] {
        const char *e = ab_env("NMZ_REPLAY_OQ");
        return !(e && std::string(e) == "0");
    }();
    return on;
}

// image size (uint2 units, before the region offsets) of one class segment's order-query arrays
struct OqLen {
    uint64_t v[4] = {0, 0, 0, 0};  // level 0, 1, 2 and samples
};
static OqLen oq_seg_len(uint32_t n) {
    OqLen l;
    if (n > OQ_BRUTE) {
        l.v[0] = oq_skew(oq_round(n, OQ_S0));
        l.v[1] = l.v[2] = oq_skew(oq_round(n, OQ_S1));
        uint32_t p2 = 1;
        while (p2 < (n + 7) / 8) p2 <<= 1;
        l.v[3] = oq_skew(p2);
    }
    return l;
}
static uint64_t oq_image_bytes(const uint64_t (&len)[4]) {
    return ((len[0] + len[1] + len[2] + len[3]) * 8 + 15) & ~15ull;
}

// Build the order-query row images after the C sort (0 < m < 2^32). A row image that fits one workgroup's LDS
// is one pass over the length classes (configs[1]: 110 KB at E = 4,096). A longer trace splits its classes into
// C-sorted sub-segments of at most OQ_SUBSEG events -- each one is a segment in its own right: every decision of
// it is (base + Cm) mod m with the same carry rule (C > ~H), just over fewer events -- and packs them into passes
// whose images fit; the kernel runs once per pass and combines the passes' statistics per seed.
constexpr uint32_t OQ_SUBSEG = 4096;
static int oq_build(nmz_replayable_plan *p, const std::vector<ClassInfo> &cls, hipStream_t st) {
    const uint32_t E = p->n_events;
    p->oq = false;
    p->oq_passes.clear();
    if (!p->mod.m32ok || E == 0) return NMZ_OK;
    uint64_t budget = OQ_LDS_MAX - OQ_TAIL_LDS;
    if (const char *e = ab_env("NMZ_REPLAY_OQ_BUDGET"))  // tests: force several passes on short traces
        budget = std::min<uint64_t>(budget, std::max<uint64_t>(4096, strtoull(e, nullptr, 10)));
    // segments: the classes whole when the whole row fits one pass, else sub-segments of <= OQ_SUBSEG events
    std::vector<ClassInfo> seg;
    {
        uint64_t len[4] = {1, 0, 0, 0};
        for (const ClassInfo &c : cls) {
            const OqLen l = oq_seg_len(c.count);
            for (int r = 0; r < 4; ++r) len[r] += l.v[r];
        }
        const bool split = oq_image_bytes(len) > budget;
        // sub-segments small enough that one always fits the budget
        uint32_t sub = OQ_SUBSEG;
        while (sub > OQ_S0) {
            const OqLen l = oq_seg_len(sub);
            const uint64_t one[4] = {1 + l.v[0], l.v[1], l.v[2], l.v[3]};
            if (oq_image_bytes(one) <= budget) break;
            sub /= 2;
        }
        for (const ClassInfo &c : cls) {
            if (!split || c.count <= sub) {
                seg.push_back(c);
                continue;
            }
            for (uint32_t lo = 0; lo < c.count; lo += sub)
                seg.push_back(ClassInfo{c.pn, c.start + lo, std::min(sub, c.count - lo)});
        }
    }
    // passes: consecutive segments while the image fits (slot 0 of every image stays free, so the read below a
    // block, unused when the count is 0, never leaves the image)
    std::vector<OqClass> oc(seg.size());
    std::vector<uint4> tbl;
    uint64_t off16 = 0;
    for (size_t c0 = 0; c0 < seg.size();) {
        uint64_t len[4] = {1, 0, 0, 0};
        size_t c1 = c0;
        for (; c1 < seg.size(); ++c1) {
            const OqLen l = oq_seg_len(seg[c1].count);
            uint64_t t[4];
            for (int r = 0; r < 4; ++r) t[r] = len[r] + l.v[r];
            if (c1 > c0 && oq_image_bytes(t) > budget) break;
            OqClass &o = oc[c1];
            o = OqClass{};
            o.pn = seg[c1].pn;
            o.start = seg[c1].start;
            o.count = seg[c1].count;
            o.pass = (uint32_t)p->oq_passes.size();
            if (o.count > OQ_BRUTE) {
                o.lv[0] = (uint32_t)len[0];
                o.lv[1] = (uint32_t)len[1];
                o.lv[2] = (uint32_t)len[2];
                o.samp = (uint32_t)len[3];
                uint32_t p2 = 1;
                while (p2 < (o.count + 7) / 8) p2 <<= 1;
                o.samp_p2 = p2;
            }
            for (int r = 0; r < 4; ++r) len[r] = t[r];
            for (uint32_t lo = 0; lo < o.count; lo += OQ_S0)
                tbl.push_back(make_uint4((uint32_t)c1, lo, std::min(OQ_S0, o.count - lo), 0));
        }
        const uint64_t rb = oq_image_bytes(len);
        if (rb > budget) return NMZ_OK;  // cannot happen with OQ_SUBSEG segments; keep the per-decision sweep
        for (size_t c = c0; c < c1; ++c) {  // regions: level 0 | level 1 | level 2 | samples
            oc[c].lv[1] += (uint32_t)len[0];
            oc[c].lv[2] += (uint32_t)(len[0] + len[1]);
            oc[c].samp += (uint32_t)(len[0] + len[1] + len[2]);
        }
        p->oq_passes.push_back(nmz_replayable_plan::OqPass{(uint32_t)c0, (uint32_t)c1, off16, (uint32_t)(rb / 16)});
        off16 += 256 * (rb / 16);
        c0 = c1;
    }
    // function attributes are per device, and contexts on several devices (or threads) build plans
    // concurrently: set them on every build (cheap) instead of behind a process-wide flag
    for (const void *f : {reinterpret_cast<const void *>(k_replayable_sweep_oq<false, false>),
                          reinterpret_cast<const void *>(k_replayable_sweep_oq<false, true>),
                          reinterpret_cast<const void *>(k_replayable_sweep_oq<true, false>),
                          reinterpret_cast<const void *>(k_replayable_sweep_oq<true, true>)})
        if (hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, (int)OQ_LDS_MAX) != hipSuccess) {
            p->oq_passes.clear();
            return NMZ_OK;  // keep the per-decision sweep
        }
    const size_t np = p->oq_passes.size();
    std::vector<uint4> passes(np);
    for (size_t i = 0; i < np; ++i)
        passes[i] = make_uint4((uint32_t)p->oq_passes[i].off16, (uint32_t)(p->oq_passes[i].off16 >> 32),
                               p->oq_passes[i].rb16, 0);
    const size_t need = Carve::bytes_for(off16, 16) + Carve::bytes_for(256 * np, 8) +
                        Carve::bytes_for(oc.size(), sizeof(OqClass)) + Carve::bytes_for(tbl.size(), 16) +
                        Carve::bytes_for(np, 16);
    NMZ_TRY(p->oq_mem.ensure(need));
    Carve cv(p->oq_mem.ptr);
    p->d_oq_blob = cv.take<uint4>(off16);
    p->d_oq_rowsum = cv.take<uint64_t>(256 * np);
    p->d_oq_classes = cv.take<OqClass>(oc.size());
    uint4 *d_tbl = cv.take<uint4>(tbl.size());
    uint4 *d_passes = cv.take<uint4>(np);
    NMZ_HIP(hipMemsetAsync(p->d_oq_blob, 0, off16 * 16, st));
    NMZ_HIP(hipMemsetAsync(p->d_oq_rowsum, 0, 256 * np * 8, st));
    NMZ_HIP(hipMemcpyAsync(p->d_oq_classes, oc.data(), oc.size() * sizeof(OqClass), hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_tbl, tbl.data(), tbl.size() * 16, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_passes, passes.data(), np * 16, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_replayable_oq_levels, dim3((unsigned)tbl.size(), 256), dim3(256), 0, st, p->d_table, E, d_tbl,
                       p->d_oq_classes, d_passes, p->d_oq_blob,
                       reinterpret_cast<unsigned long long *>(p->d_oq_rowsum));
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipStreamSynchronize(st));  // the host vectors above are pageable
    p->oq = true;
    return NMZ_OK;
}

static size_t seed_scratch_bytes(uint64_t S) {
    uint64_t max_units = S / REPLAY_SEEDS_PER_UNIT_MIN + 257;
    return Carve::bytes_for(S, 8) * 2 + Carve::bytes_for(S, 4) + Carve::bytes_for(BUCKET_SMALL_U32, 4) +
           Carve::bytes_for(bucket_hist_u32(S), 4) + Carve::bytes_for(max_units, 16) + Carve::bytes_for(4, 4);
}

static size_t partial_bytes(uint64_t S, uint32_t E, int U, uint32_t ec) {
    const uint64_t units = S / (64 * (uint64_t)U) + 257;
    const uint64_t chunks = (E + ec - 1) / ec;
    return Carve::bytes_for(units * 64 * U * chunks, 16);
}

struct SeedScratch {
    uint64_t *h0;
    Buckets b;
    uint32_t *counter;
};

static SeedScratch carve_seed_scratch(void *p, uint64_t S) {
    Carve cv(p);
    SeedScratch s;
    s.h0 = cv.take<uint64_t>(S);
    s.b.sorted_h0 = cv.take<uint64_t>(S);
    s.b.sorted_idx = cv.take<uint32_t>(S);
    buckets_small(cv.take<uint32_t>(BUCKET_SMALL_U32), s.b);
    s.b.hist = cv.take<uint32_t>(bucket_hist_u32(S));
    s.b.units = cv.take<uint4>(S / REPLAY_SEEDS_PER_UNIT_MIN + 257);
    s.counter = cv.take<uint32_t>(4);
    return s;
}

// enqueue the sweep for device-resident seeds
// Stats for every seed.
// Seeds: the CSR d_soff / d_sbytes, or (d_soff == nullptr) the decimal strings of dec_lo .. dec_lo + S - 1.
// the wavelet-tree sweep runs this plan's sweeps
static bool use_wt(const nmz_replayable_plan *p) {
    return p->wt.on && (replay_oq_enabled() || p->mod.kind != MOD_FAST);
}

// top-k on the wavelet-tree path: candidates above the k-th largest workgroup maximum (NMZ_WT_TOPK=0: the general
// selection, for A/B runs)
static bool wt_topk_enabled() {
    static const bool on = [] {
        const char *e = ab_env("NMZ_WT_TOPK");
        return !(e && std::string(e) == "0");
    }();
    return on;
}

}  // namespace nmz

// A prepared seed set (nmz_replayable_seeds_create): the seeds' prefix hashes, bucketed by row at the statistics
// kernels' granularity, and the row histogram (the per-decision sweeps bucket the hashes again at theirs)
struct nmz_replayable_seeds {
    nmz_ctx *ctx = nullptr;
    uint64_t S = 0;
    nmz::DevBuf mem;
    nmz::SeedScratch sc{};
    uint32_t *hist = nullptr;  // [bucket_hist_u32(S)] the prefix kernel's rows of bucket counts
};

namespace nmz {

static int replayable_stats(nmz_replayable_plan *p, hipStream_t st, const uint32_t *d_soff,
                            const uint8_t *d_sbytes, uint64_t S, nmz_sched_stats *d_stats, uint64_t dec_lo = 0,
                            void *wt_topk_scratch = nullptr, uint32_t k = 0,
                            const nmz_replayable_seeds *pre = nullptr) {
    if (S == 0) return NMZ_OK;
    const uint32_t E = p->n_events;
    if (E == 0 || p->mod.kind == MOD_ZERO) {
        hipLaunchKernelGGL(k_stats_constant, dim3(ceil_div(S, 256)), dim3(256), 0, st, S, E, d_stats);
        NMZ_HIP(hipGetLastError());
        return NMZ_OK;
    }
    const bool stats_kernel = use_wt(p) || (p->oq && (replay_oq_enabled() || p->mod.kind != MOD_FAST));
    SeedScratch sc;
    if (pre && stats_kernel) {
        sc = pre->sc;  // bucketed already
    } else {
        NMZ_CHECK(S <= p->max_seeds, "more seeds than the plan was created for");
        sc = carve_seed_scratch(p->seed_scratch.ptr, p->max_seeds);
        if (pre) {  // a per-decision sweep of prepared seeds: their hashes and row counts, bucketed here
            NMZ_HIP(hipMemcpyAsync(sc.b.hist, pre->hist, bucket_hist_u32(S) * sizeof(uint32_t),
                                   hipMemcpyDeviceToDevice, st));
            sc.h0 = pre->sc.h0;
        } else if (d_soff) {
            hipLaunchKernelGGL(k_seed_prefix, dim3(ceil_div(S, BUCKET_BLK)), dim3(256), 0, st, d_soff, d_sbytes, S,
                               sc.h0, sc.b.hist);
        } else {
            hipLaunchKernelGGL(k_seed_prefix_decimal, dim3(ceil_div(S, BUCKET_BLK)), dim3(256), 0, st, dec_lo, S,
                               sc.h0, sc.b.hist);
        }
    }
    const bool bucketed = pre && stats_kernel;
    const int U = replay_u();
    const uint32_t per_unit = 64u * (uint32_t)U;
    const uint64_t max_units = S / per_unit + 256;
    if (use_wt(p)) {
        if (!bucketed) NMZ_TRY(bucket_seeds_counted(st, sc.h0, S, OQ_WG, sc.b, sc.counter));
        return wt_sweep(p->wt, p->ctx, st, sc.b, p->d_table, E, p->mod, d_stats, S, wt_topk_scratch, k);
    }
    if (p->oq && (replay_oq_enabled() || p->mod.kind != MOD_FAST)) {
        if (!bucketed) NMZ_TRY(bucket_seeds_counted(st, sc.h0, S, OQ_WG, sc.b, sc.counter));
        KernelTimer kt(p->ctx, st, "replayable_sweep");
        unsigned long long *span = kt.span();
        const bool big = p->mod.m32 >= 0x80000000u;
        for (size_t i = 0; i < p->oq_passes.size(); ++i) {
            const nmz_replayable_plan::OqPass &ps = p->oq_passes[i];
            auto kern = big ? (i ? k_replayable_sweep_oq<true, true> : k_replayable_sweep_oq<true, false>)
                            : (i ? k_replayable_sweep_oq<false, true> : k_replayable_sweep_oq<false, false>);
            hipLaunchKernelGGL(kern, dim3(256), dim3(OQ_WG), ps.rb16 * 16u + OQ_TAIL_LDS, st, sc.b.offset,
                               sc.b.sorted_h0, sc.b.sorted_idx, p->d_table, E, p->d_oq_blob + ps.off16, ps.rb16,
                               reinterpret_cast<const unsigned long long *>(p->d_oq_rowsum + 256 * i),
                               p->d_oq_classes + ps.c0, ps.c1 - ps.c0, p->mod.m32, p->mod.mu, p->mod.m_k64, d_stats,
                               span);
        }
        NMZ_HIP(hipGetLastError());
        return NMZ_OK;
    }
    NMZ_TRY(bucket_seeds_counted(st, sc.h0, S, p->mod.kind == MOD_FAST ? per_unit : 64, sc.b, sc.counter));
    if (p->mod.kind == MOD_FAST) {
        const uint32_t ec = replay_ec();
        const uint32_t n_chunks = (E + ec - 1) / ec;
        NMZ_TRY(p->partial.ensure(partial_bytes(p->max_seeds, E, U, ec)));
        const uint64_t stride = (p->max_seeds / per_unit + 257) * (uint64_t)per_unit;
        // fold the u32 partial sums every 2^f groups of 4 events, (4 << f)(m - 1) + 3(m - 1) < 2^32
        uint32_t fold_mask = 0;
        while (fold_mask < 15 && ((uint64_t)(4 * (fold_mask + 1) * 2 + 3)) * (p->mod.m - 1) < (1ull << 32))
            fold_mask = fold_mask * 2 + 1;
        const unsigned grid = (unsigned)std::min<uint64_t>(p->ctx->n_cu * (uint64_t)replay_wg_per_cu(),
                                                           ceil_div(max_units * n_chunks, 4));
        {
            KernelTimer kt(p->ctx, st, "replayable_sweep");
#define NMZ_K1(UU)                                                                                                   \
    hipLaunchKernelGGL((replay_key_mode() == 1 ? k_replayable_sweep_fast<UU, 1> : k_replayable_sweep_fast<UU, 0>), dim3(grid), dim3(256), 0, st, sc.b.units, sc.b.n_units,          \
                       sc.b.sorted_h0, p->d_table, E, p->d_classes, p->n_classes, p->mod.m, p->mod.mu, p->mod.m_k64, ec,        \
                       n_chunks, fold_mask, sc.counter, p->partial.as<uint4>(), stride)
            if (U == 2) NMZ_K1(2); else if (U == 8) NMZ_K1(8); else NMZ_K1(4);
#undef NMZ_K1
        }
        const unsigned mgrid = ceil_div(max_units * per_unit, 256);
        if (U == 2)
            hipLaunchKernelGGL(k_replayable_merge<2>, dim3(mgrid), dim3(256), 0, st, sc.b.units, sc.b.n_units,
                               sc.b.sorted_idx, p->partial.as<uint4>(), stride, n_chunks, d_stats);
        else if (U == 8)
            hipLaunchKernelGGL(k_replayable_merge<8>, dim3(mgrid), dim3(256), 0, st, sc.b.units, sc.b.n_units,
                               sc.b.sorted_idx, p->partial.as<uint4>(), stride, n_chunks, d_stats);
        else
            hipLaunchKernelGGL(k_replayable_merge<4>, dim3(mgrid), dim3(256), 0, st, sc.b.units, sc.b.n_units,
                               sc.b.sorted_idx, p->partial.as<uint4>(), stride, n_chunks, d_stats);
    } else {
        KernelTimer kt(p->ctx, st, "replayable_sweep");
        const uint64_t units64 = S / 64 + 256;
        hipLaunchKernelGGL(k_replayable_sweep_general, dim3(ceil_div(units64, 4)), dim3(256), 0, st,
                           sc.b.units, sc.b.n_units, sc.b.sorted_h0, sc.b.sorted_idx, p->d_table, E,
                           p->d_classes, p->n_classes, p->mod.m, d_stats);
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// Optional top-k (k > 0): by (sum_delay desc, seed asc) over the seeds' stats (n_fault = 0), seed =
// seed0 + seed index. (A merge kernel with the first selection level fused in measured 66 us against
// 21 + 29 us for k_replayable_merge + k_topk_chunk at 2^20 seeds, so the levels stay separate.)
static int replayable_run_on(nmz_replayable_plan *p, hipStream_t st, const uint32_t *d_soff, const uint8_t *d_sbytes,
                             uint64_t S, nmz_sched_stats *d_stats, uint64_t seed0, uint32_t k, nmz_topk_entry *d_topk,
                             uint64_t dec_lo, const nmz_replayable_seeds *pre);

static int replayable_run(nmz_replayable_plan *p, hipStream_t st, const uint32_t *d_soff, const uint8_t *d_sbytes,
                          uint64_t S, nmz_sched_stats *d_stats, uint64_t seed0 = 0, uint32_t k = 0,
                          nmz_topk_entry *d_topk = nullptr, uint64_t dec_lo = 0,
                          const nmz_replayable_seeds *pre = nullptr) {
    nmz_replayable_plan::Use *u = nullptr;
    for (auto &x : p->uses)
        if (x.st == st) u = &x;
    if (!u) {  // the plan's first sweep on this stream: the stream waits for the build (a no-op once it is done)
        hipEvent_t ev;
        NMZ_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        p->uses.push_back({st, ev});
        u = &p->uses.back();
        if (p->built && st != p->ctx->stream) NMZ_HIP(hipStreamWaitEvent(st, p->built, 0));
    }
    const int rc = replayable_run_on(p, st, d_soff, d_sbytes, S, d_stats, seed0, k, d_topk, dec_lo, pre);
    NMZ_HIP(hipEventRecord(u->ev, st));
    return rc;
}

// the plan's build and every sweep enqueued with it are done: its pooled buffers may go back to the context
static void plan_wait_uses(nmz_replayable_plan *p) {
    for (auto &u : p->uses) {
        (void)hipEventSynchronize(u.ev);
        (void)hipEventDestroy(u.ev);
    }
    p->uses.clear();
    if (p->built) {
        (void)hipEventSynchronize(p->built);
        (void)hipEventDestroy(p->built);
        p->built = nullptr;
    } else {
        (void)hipStreamSynchronize(p->ctx->stream);
    }
}

static int replayable_run_on(nmz_replayable_plan *p, hipStream_t st, const uint32_t *d_soff, const uint8_t *d_sbytes,
                             uint64_t S, nmz_sched_stats *d_stats, uint64_t seed0, uint32_t k, nmz_topk_entry *d_topk,
                             uint64_t dec_lo, const nmz_replayable_seeds *pre) {
    NMZ_CHECK(k <= 256, "top-k supports k <= 256");
    NMZ_CHECK(k == 0 || d_topk, "d_topk is NULL");
    // the wavelet-tree sweep's own candidates (k <= 64; more than one general-selection list, so that the gated
    // fallback has its merge levels): the general selection runs only when they overflow
    const bool fused = k && k <= 64 && S > 0 && use_wt(p) && wt_topk_enabled();
    if (fused) {
        NMZ_TRY(p->wt_topk.ensure(wt_topk_scratch_bytes(S)));  // the sweep zeroes its candidate counter
    }
    NMZ_TRY(replayable_stats(p, st, d_soff, d_sbytes, S, d_stats, dec_lo, fused ? p->wt_topk.ptr : nullptr, k, pre));
    if (fused) {  // the seeds' order of the sweep that ran (the prepared set's, or this plan's own bucketing)
        const uint32_t *sidx = pre ? pre->sc.b.sorted_idx
                                   : carve_seed_scratch(p->seed_scratch.ptr, p->max_seeds).b.sorted_idx;
        return wt_topk(st, p->wt_topk.ptr, sidx, S, seed0, k, d_topk);
    }
    if (k) {
        NMZ_TRY(p->topk_lists.ensure(topk_scratch_entries(S, k) * sizeof(nmz_topk_entry)));
        NMZ_TRY(topk_select(st, d_stats, S, seed0, k, p->topk_lists.as<nmz_topk_entry>(), d_topk));
    }
    return NMZ_OK;
}

// the caller holds the plan's context: the buffers go back to the context's pool, where the next plan may write
// them at once, so wait for the work still reading them -- the build and the sweeps on every stream the plan was
// used on
static void plan_destroy_locked(nmz_replayable_plan *plan) {
    plan_wait_uses(plan);
    plan->plan_mem.release();
    plan->seed_scratch.release();
    plan->partial.release();
    plan->topk_lists.release();
    plan->oq_mem.release();
    plan->wt.mem.release();
    plan->wt.aux.release();
    plan->wt_topk.release();
    delete plan;
}

static int plan_create(nmz_ctx *ctx, const uint32_t *hint_off, const uint8_t *hint_bytes, uint32_t E,
                       int64_t max_interval, uint64_t max_seeds, nmz_replayable_plan **out, bool async = false) {
    NMZ_CHECK(ctx && out, "NULL argument");
    NMZ_CHECK(E == 0 || hint_off, "hint_off is NULL");
    *out = nullptr;
    auto *p = new nmz_replayable_plan();
    p->ctx = ctx;
    for (DevBuf *b : {&p->seed_scratch, &p->partial, &p->topk_lists, &p->plan_mem, &p->oq_mem, &p->wt.mem,
                      &p->wt.aux, &p->wt_topk})
        b->pool = &ctx->pool;
    p->n_events = E;
    p->max_interval = max_interval;
    p->mod = make_mod((uint64_t)max_interval);  // uint64(r.MaxInterval), replayablepolicy.go:110
    p->max_seeds = max_seeds;
    hipStream_t st = ctx->stream;

    // length classes (stable, so original order is kept inside a class): a counting sort by hint length (a
    // comparison sort of 4,096 hints was ~100 us of the plan's host time)
    std::vector<uint32_t> perm(E);
    uint32_t maxlen = 0;
    for (uint32_t e = 0; e < E; ++e) maxlen = std::max(maxlen, hint_off[e + 1] - hint_off[e]);
    if (maxlen > 4 * (uint64_t)E + 4096) {  // a few very long hints: a comparison sort
        std::iota(perm.begin(), perm.end(), 0u);
        std::stable_sort(perm.begin(), perm.end(), [&](uint32_t a, uint32_t b) {
            return hint_off[a + 1] - hint_off[a] < hint_off[b + 1] - hint_off[b];
        });
    } else {
        std::vector<uint32_t> pos((size_t)maxlen + 2, 0);
        for (uint32_t e = 0; e < E; ++e) ++pos[hint_off[e + 1] - hint_off[e] + 1];
        for (size_t l = 1; l < pos.size(); ++l) pos[l] += pos[l - 1];
        for (uint32_t e = 0; e < E; ++e) perm[pos[hint_off[e + 1] - hint_off[e]]++] = e;
    }
    std::vector<ClassInfo> cls;  // runs of equal length in the length-sorted order (P^len once per class)
    for (uint32_t i = 0, prev = 0; i < E; ++i) {
        const uint32_t e = perm[i];
        const uint32_t len = hint_off[e + 1] - hint_off[e];
        if (cls.empty() || len != prev) {
            cls.push_back(ClassInfo{fnv_pow(len), i, 0});
            prev = len;
        }
        cls.back().count++;
    }
    p->n_classes = (uint32_t)cls.size();
    const uint64_t nbytes = E ? hint_off[E] : 0;

    // the wavelet-tree plan kernel computes and C-sorts the table itself when every class fits one of its segments:
    // its segment descriptors and zeroed row sums go up with the plan's inputs, and it zeroes the seed scratch's
    // counters itself -- one upload and one launch. (NMZ_WT_FUSED=0 takes the separate kernels always: parity tests
    // and A/B runs.)
    std::vector<WtClass> woc;
    const bool fused = E && !(ab_env("NMZ_WT_FUSED") && atoi(ab_env("NMZ_WT_FUSED")) == 0) &&
                       wt_layout(p->wt, ctx, E, cls.data(), (uint32_t)cls.size(), p->mod, true, woc);
    size_t need = Carve::bytes_for(cls.size() + 1, sizeof(ClassInfo)) + Carve::bytes_for((size_t)256 * E + 1, 16) +
                  Carve::bytes_for(E + 1, 4) * 2 + Carve::bytes_for(nbytes + 1, 1);
    if (fused) need += Carve::bytes_for(woc.size(), sizeof(WtClass)) + Carve::bytes_for(256, 8);
    int rc = p->plan_mem.ensure(need);
    SeedScratch sc0{};
    const bool seeds = E && p->mod.kind != MOD_ZERO;
    if (rc == NMZ_OK && seeds) {
        rc = p->seed_scratch.ensure(seed_scratch_bytes(max_seeds));
        if (rc == NMZ_OK) {  // the work-item counter starts at zero (k_bucket_scatter re-zeroes it)
            sc0 = carve_seed_scratch(p->seed_scratch.ptr, max_seeds);
            if (!fused && hipMemsetAsync(sc0.counter, 0, 4 * sizeof(uint32_t), st) != hipSuccess)
                rc = fail(NMZ_EHIP, "hipMemsetAsync of the seed scratch failed");
        }
    }
    if (rc != NMZ_OK) {
        (void)hipStreamSynchronize(st);
        p->plan_mem.release();
        p->seed_scratch.release();
        delete p;
        return rc;
    }
    // the small inputs first (one contiguous region, packed in the context's pinned staging at the same offsets:
    // one asynchronous upload), then the table
    Carve cv(p->plan_mem.ptr);
    p->d_classes = cv.take<ClassInfo>(cls.size() + 1);
    uint32_t *d_perm = cv.take<uint32_t>(E + 1);
    uint32_t *d_hoff = p->d_hoff = cv.take<uint32_t>(E + 1);
    uint8_t *d_hbytes = p->d_hbytes = cv.take<uint8_t>(nbytes + 1);
    WtClass *d_wcls = fused ? cv.take<WtClass>(woc.size()) : nullptr;
    unsigned long long *d_rowsum = fused ? cv.take<unsigned long long>(256) : nullptr;
    const size_t in_bytes = (size_t)(reinterpret_cast<char *>(cv.take<uint4>(0)) - reinterpret_cast<char *>(p->plan_mem.ptr));
    p->d_table = cv.take<uint4>((size_t)256 * E + 1);
    auto cleanup = [&](int code) {
        (void)hipStreamSynchronize(st);  // pooled buffers: no work may still use them
        p->plan_mem.release();
        p->seed_scratch.release();
        p->partial.release();
        p->topk_lists.release();
        p->oq_mem.release();
        p->wt.mem.release();
        p->wt.aux.release();
        p->wt_topk.release();
        delete p;
        return code;
    };
    if (E) {
        HostPin &pin = ctx->pin[0];
        if (pin.ensure(in_bytes) != NMZ_OK) return cleanup(NMZ_ENOMEM);
        {
            char *h = static_cast<char *>(pin.ptr);
            auto at = [&](const void *d) { return h + (static_cast<const char *>(d) - static_cast<char *>(p->plan_mem.ptr)); };
            std::memcpy(at(p->d_classes), cls.data(), cls.size() * sizeof(ClassInfo));
            std::memcpy(at(d_perm), perm.data(), (size_t)E * 4);
            std::memcpy(at(d_hoff), hint_off, (size_t)(E + 1) * 4);
            if (nbytes) std::memcpy(at(d_hbytes), hint_bytes, nbytes);
            if (fused) {
                std::memcpy(at(d_wcls), woc.data(), woc.size() * sizeof(WtClass));
                std::memset(at(d_rowsum), 0, 256 * 8);
            }
        }
        if (hipMemcpyAsync(p->plan_mem.ptr, pin.ptr, in_bytes, hipMemcpyHostToDevice, st) || pin.mark(st))
            return cleanup(fail(NMZ_EHIP, "plan upload failed"));
        if (fused) {
            const WtPlanHints hz{d_hoff, d_hbytes, d_perm, p->d_table,
                                 nullptr, 0u, seeds ? sc0.counter : nullptr, seeds ? 4u : 0u};
            const int wrc = wt_launch(p->wt, p->d_table, E, p->mod, st, &hz, d_wcls, d_rowsum, !async);
            if (wrc != NMZ_OK) return cleanup(wrc);
        }
        if (!p->wt.on) {
            // unsorted table into scratch (the context's, grow-only: no free, so no device sync), then the
            // per-(L, class) C sort into place
            DevBuf &tmp = ctx->buf[10];
            if (tmp.ensure((size_t)256 * E * sizeof(uint4)) != NMZ_OK) return cleanup(NMZ_ENOMEM);
            hipLaunchKernelGGL(k_replayable_table, dim3(E), dim3(256), 0, st, d_hoff, d_hbytes, d_perm, E, p->mod.m,
                               p->mod.m32ok ? 1 : 0, tmp.as<uint4>());
            uint32_t max_class = 0;
            for (const ClassInfo &c : cls) max_class = std::max(max_class, c.count);
            bool bad = false;
            if (max_class <= SEG_SORT_MAX && !ab_env("NMZ_REPLAY_RANKSORT")) {  // LDS bitonic sort per segment
                hipLaunchKernelGGL(k_replayable_table_segsort, dim3(p->n_classes, 256), dim3(1024), 0, st,
                                   tmp.as<uint4>(), p->d_classes, E, p->d_table);
                // no sync when the order-query images follow: oq_build synchronises after its kernels
                bad = hipGetLastError() != hipSuccess ||
                      (!p->mod.m32ok && hipStreamSynchronize(st) != hipSuccess);
            } else if (max_class <= 16384) {  // O(n^2) rank sort on the device
                hipLaunchKernelGGL(k_replayable_table_sort, dim3(ceil_div(E, 256), 256), dim3(256), 0, st,
                                   tmp.as<uint4>(), p->d_classes, p->n_classes, E, p->d_table);
                bad = hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess;
            } else {  // very large classes: sort the segments on the host
                std::vector<uint4> h((size_t)256 * E);
                bad = hipGetLastError() != hipSuccess ||
                      hipMemcpyAsync(h.data(), tmp.ptr, h.size() * sizeof(uint4), hipMemcpyDeviceToHost, st) !=
                          hipSuccess ||
                      hipStreamSynchronize(st) != hipSuccess;
                if (!bad) {
                    auto key = [](const uint4 &q) { return ((uint64_t)q.y << 32) | q.x; };
                    for (uint32_t L = 0; L < 256; ++L)
                        for (const ClassInfo &c : cls)
                            std::stable_sort(h.begin() + (size_t)L * E + c.start,
                                             h.begin() + (size_t)L * E + c.start + c.count,
                                             [&](const uint4 &a, const uint4 &b) { return key(a) < key(b); });
                    bad = hipMemcpyAsync(p->d_table, h.data(), h.size() * sizeof(uint4), hipMemcpyHostToDevice, st) !=
                              hipSuccess ||
                          hipStreamSynchronize(st) != hipSuccess;
                }
            }
            if (bad)
                return cleanup(fail(NMZ_EHIP, "plan table kernel failed"));
            // wavelet-tree images (the default sweep when they fit), else the order-query images
            int orc = wt_build(p->wt, ctx, p->d_table, E, cls.data(), (uint32_t)cls.size(), p->mod, st);
            if (orc != NMZ_OK) return cleanup(orc);
            if (!p->wt.on) orc = oq_build(p, cls, st);
            if (orc != NMZ_OK) return cleanup(orc);
        }
        // the plan is complete before it is returned (sweeps may run on any stream), or, from the asynchronous
        // entry point with the wavelet-tree plan kernel, enqueued: sweeps on other streams wait for `built`
        if (!p->oq && !p->wt.on && hipStreamSynchronize(st) != hipSuccess)
            return cleanup(fail(NMZ_EHIP, "plan build failed"));
    }
    if (hipEventCreateWithFlags(&p->built, hipEventDisableTiming) != hipSuccess) {
        p->built = nullptr;
        return cleanup(fail(NMZ_EHIP, "hipEventCreate failed"));
    }
    if (hipEventRecord(p->built, st) != hipSuccess) return cleanup(fail(NMZ_EHIP, "hipEventRecord failed"));
    *out = p;
    return NMZ_OK;
}

// the caller holds ctx (nmz_replayable_seeds_create, nmz_replayable_sweep_traces)
static int seeds_create_locked(nmz_ctx *ctx, const uint32_t *d_seed_off, const uint8_t *d_seed_bytes, uint64_t n_seeds,
                               uint64_t dec_lo, nmz_replayable_seeds **out) {
    *out = nullptr;
    auto *s = new nmz_replayable_seeds();
    s->ctx = ctx;
    s->S = n_seeds;
    s->mem.pool = &ctx->pool;  // a stream of seed sets of one size reuses one buffer (no hipMalloc per set)
    hipStream_t st = ctx->stream;
    const int rc = s->mem.ensure(seed_scratch_bytes(n_seeds) + Carve::bytes_for(bucket_hist_u32(n_seeds), 4));
    if (rc != NMZ_OK) {
        delete s;
        return rc;
    }
    s->sc = carve_seed_scratch(s->mem.ptr, n_seeds);
    s->hist = reinterpret_cast<uint32_t *>(static_cast<char *>(s->mem.ptr) + seed_scratch_bytes(n_seeds));
    auto fail_hip = [&]() {
        (void)hipStreamSynchronize(st);
        s->mem.release();
        delete s;
        return fail(NMZ_EHIP, "seed set build failed");
    };
    if (hipMemsetAsync(s->sc.counter, 0, 4 * sizeof(uint32_t), st) != hipSuccess) return fail_hip();
    if (d_seed_off)
        hipLaunchKernelGGL(k_seed_prefix, dim3(ceil_div(n_seeds, BUCKET_BLK)), dim3(256), 0, st, d_seed_off,
                           d_seed_bytes, n_seeds, s->sc.h0, s->sc.b.hist);
    else
        hipLaunchKernelGGL(k_seed_prefix_decimal, dim3(ceil_div(n_seeds, BUCKET_BLK)), dim3(256), 0, st, dec_lo,
                           n_seeds, s->sc.h0, s->sc.b.hist);
    if (hipGetLastError() != hipSuccess ||
        hipMemcpyAsync(s->hist, s->sc.b.hist, bucket_hist_u32(n_seeds) * sizeof(uint32_t), hipMemcpyDeviceToDevice,
                       st) != hipSuccess ||
        bucket_seeds_counted(st, s->sc.h0, n_seeds, OQ_WG, s->sc.b, s->sc.counter) != NMZ_OK ||
        hipStreamSynchronize(st) != hipSuccess)
        return fail_hip();
    *out = s;
    return NMZ_OK;
}

static void seeds_destroy_locked(nmz_replayable_seeds *seeds) {
    (void)hipDeviceSynchronize();  // sweeps on any stream may still read the set (its buffer goes to the pool)
    seeds->mem.release();
    delete seeds;
}

}  // namespace nmz

using namespace nmz;

extern "C" {
#ifdef OQ_TRACE
int nmz_debug_oq_trace(unsigned long long *out) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(nmz::g_oq_trace), sizeof(nmz::g_oq_trace)) == hipSuccess ? 0 : -1;
}
#endif

int nmz_replayable_plan_create(nmz_ctx *ctx, const uint32_t *hint_off, const uint8_t *hint_bytes,
                               uint32_t n_events, int64_t max_interval_ns, uint64_t max_seeds,
                               nmz_replayable_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return plan_create(ctx, hint_off, hint_bytes, n_events, max_interval_ns, max_seeds, out);
}

int nmz_replayable_plan_create_async(nmz_ctx *ctx, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                     uint32_t n_events, int64_t max_interval_ns, uint64_t max_seeds,
                                     nmz_replayable_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return plan_create(ctx, hint_off, hint_bytes, n_events, max_interval_ns, max_seeds, out, true);
}

int nmz_replayable_plan_destroy(nmz_replayable_plan *plan) {
    if (!plan) return NMZ_OK;
    {
        CtxGuard g(plan->ctx);
        plan_destroy_locked(plan);
    }
    return NMZ_OK;
}

int nmz_replayable_plan_kernel(const nmz_replayable_plan *plan) {
    if (!plan) return -1;
    return plan->wt.on ? 2 : plan->oq ? 1 : 0;
}

int nmz_replayable_sweep_dev(nmz_replayable_plan *plan, const uint32_t *d_seed_off, const uint8_t *d_seed_bytes,
                             uint64_t n_seeds, nmz_sched_stats *d_stats, void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = stream ? (hipStream_t)stream : plan->ctx->stream;
    return replayable_run(plan, st, d_seed_off, d_seed_bytes, n_seeds, d_stats);
}

int nmz_replayable_sweep_topk_dev(nmz_replayable_plan *plan, const uint32_t *d_seed_off, const uint8_t *d_seed_bytes,
                                  uint64_t n_seeds, uint64_t seed0, uint32_t k, nmz_sched_stats *d_stats,
                                  nmz_topk_entry *d_topk, void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = stream ? (hipStream_t)stream : plan->ctx->stream;
    return replayable_run(plan, st, d_seed_off, d_seed_bytes, n_seeds, d_stats, seed0, k, d_topk);
}

int nmz_replayable_seeds_create(nmz_ctx *ctx, const uint32_t *d_seed_off, const uint8_t *d_seed_bytes, uint64_t n_seeds,
                                uint64_t dec_lo, nmz_replayable_seeds **out) {
    NMZ_CHECK(ctx != nullptr && out != nullptr, "NULL argument");
    NMZ_CHECK(n_seeds >= 1 && n_seeds < (1ULL << 32), "1 <= n_seeds < 2^32");
    NMZ_CHECK(!d_seed_off || d_seed_bytes, "d_seed_bytes is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    return seeds_create_locked(ctx, d_seed_off, d_seed_bytes, n_seeds, dec_lo, out);
}

int nmz_replayable_seeds_destroy(nmz_replayable_seeds *seeds) {
    if (!seeds) return NMZ_OK;
    {
        CtxGuard g(seeds->ctx);
        seeds_destroy_locked(seeds);
    }
    return NMZ_OK;
}

#ifndef NMZ_TRACES_ONE_STREAM
#define NMZ_TRACES_ONE_STREAM 0
#endif
#ifndef NMZ_TRACES_DEFAULT_MODE
#define NMZ_TRACES_DEFAULT_MODE 4
#endif
int nmz_replayable_sweep_traces(nmz_ctx *ctx, uint32_t n_traces, const uint32_t *const *hint_off,
                                const uint8_t *const *hint_bytes, const uint32_t *n_events, int64_t max_interval_ns,
                                uint64_t seed_lo, uint64_t n_seeds, uint32_t k, nmz_topk_entry *topk) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_traces == 0 || (hint_off && hint_bytes && n_events && topk), "NULL argument");
    NMZ_CHECK(k >= 1 && k <= 256, "1 <= k <= 256");
    NMZ_CHECK(n_seeds >= 1 && n_seeds < (1ULL << 32), "1 <= n_seeds < 2^32");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0) return NMZ_OK;
    // the pipeline's resources: the private second context (plans alternate between the two contexts' streams, so
    // one trace's build overlaps the previous trace's), two sweep streams, the stats / top-k buffers per slot
    if (!ctx->helper) NMZ_TRY(nmz_open(ctx->device, &ctx->helper));
    for (int i = 0; i < 2; ++i)
        if (!ctx->sweep_st[i]) NMZ_HIP(hipStreamCreateWithFlags(&ctx->sweep_st[i], hipStreamNonBlocking));
    for (int i = 0; i < 3; ++i)
        if (!ctx->sweep_ev[i]) NMZ_HIP(hipEventCreateWithFlags(&ctx->sweep_ev[i], hipEventDisableTiming));
    const uint64_t S = n_seeds;
    const size_t st_bytes = Carve::bytes_for(S, sizeof(nmz_sched_stats)), tk_bytes = Carve::bytes_for(k, sizeof(nmz_topk_entry));
    NMZ_TRY(ctx->buf[11].ensure(2 * (st_bytes + tk_bytes)));
    NMZ_TRY(ctx->tkpin.ensure(3 * (size_t)k * sizeof(nmz_topk_entry)));
    Carve cv(ctx->buf[11].ptr);
    nmz_sched_stats *d_st[2] = {cv.take<nmz_sched_stats>(S), cv.take<nmz_sched_stats>(S)};
    nmz_topk_entry *d_tk[2] = {cv.take<nmz_topk_entry>(k), cv.take<nmz_topk_entry>(k)};
    nmz_topk_entry *h_tk = static_cast<nmz_topk_entry *>(ctx->tkpin.ptr);
    nmz_replayable_seeds *ss = nullptr;
    NMZ_TRY(seeds_create_locked(ctx, nullptr, nullptr, S, seed_lo, &ss));
    nmz_ctx *ctxs[2] = {ctx, ctx->helper};
    std::vector<nmz_replayable_plan *> plans(n_traces, nullptr);
    const int mode = [] {
        const char *e = ab_env("NMZ_TRACES_MODE");
        return e && e[0] >= '0' && e[0] <= '5' ? e[0] - '0' : NMZ_TRACES_DEFAULT_MODE;
    }();
    auto make = [&](uint32_t j) {
        // mode 4: every build on the helper context's stream, every sweep on ctx's: a two-stage pipeline
        nmz_ctx *bc = mode >= 4 ? ctx->helper : ctxs[j % 2];
        return plan_create(bc, hint_off[j], hint_bytes[j], n_events[j], max_interval_ns, S, &plans[j], true);
    };
    auto finish = [&](uint32_t j) -> int {
        const int r = hipEventSynchronize(ctx->sweep_ev[j % 3]) == hipSuccess ? NMZ_OK
                                                                               : fail(NMZ_EHIP, "sweep failed");
        std::memcpy(topk + (size_t)j * k, h_tk + (size_t)(j % 3) * k, (size_t)k * sizeof(nmz_topk_entry));
        plan_destroy_locked(plans[j]);
        plans[j] = nullptr;
        return r;
    };
    // trace i + 2's build is enqueued while trace i sweeps; trace i's top-k comes back while trace i + 1 sweeps
    constexpr uint32_t AHEAD = 2;
    int rc = NMZ_OK;
    for (uint32_t j = 0; j < std::min(AHEAD, n_traces) && rc == NMZ_OK; ++j) rc = make(j);
    // The schedule (NMZ_TRACES_MODE, A/B). 4, the default: a two-stage pipeline -- every plan build on the helper
    // context's stream, two traces ahead, every sweep (+ top-k + its copy to the host) on ctx's stream behind the
    // build it waits for, trace i - 1's top-k read once trace i's sweep is enqueued: 0.153-0.155 ms per trace over
    // 64 traces, against 0.154-0.156 for the Python-driven stream in the same process (profiles/r05/traces_mode_ab).
    // 1: trace i sweeps on the stream its plan was built on, trace i + 2's build behind that sweep (two streams,
    // each serial): 0.165. 2: 1 with trace i's top-k read after trace i + 1's sweep. 3: the Python loop's own
    // four-stream schedule (builds on the two contexts' streams, sweeps on two more): 0.185. 0: builds and sweeps on
    // four streams, lag 2 (round 4: 0.188). 5: 4 with the sweeps alternating over two streams.
    const bool same_stream = mode == 1 || mode == 2;
    const uint32_t lag = (mode >= 2) ? 1 : 2;
    for (uint32_t i = 0; i < n_traces && rc == NMZ_OK; ++i) {
        if (!same_stream && i + AHEAD < n_traces) rc = make(i + AHEAD);
        if (rc != NMZ_OK) break;
        hipStream_t st = mode == 4   ? ctx->stream
                         : mode == 5 ? (i % 2 ? ctx->sweep_st[0] : ctx->stream)
                         : same_stream ? ctxs[i % 2]->stream
                                       : ctx->sweep_st[NMZ_TRACES_ONE_STREAM ? 0 : i % 2];
        rc = replayable_run(plans[i], st, nullptr, nullptr, S, d_st[i % 2], seed_lo, k, d_tk[i % 2], 0, ss);
        if (rc != NMZ_OK) break;
        if (hipMemcpyAsync(h_tk + (size_t)(i % 3) * k, d_tk[i % 2], (size_t)k * sizeof(nmz_topk_entry),
                           hipMemcpyDeviceToHost, st) != hipSuccess ||
            hipEventRecord(ctx->sweep_ev[i % 3], st) != hipSuccess) {
            rc = fail(NMZ_EHIP, "top-k copy failed");
            break;
        }
        if (same_stream && i + AHEAD < n_traces) rc = make(i + AHEAD);
        if (rc != NMZ_OK) break;
        // two traces stay in flight: waiting for the previous one here would hold back the next plan builds
        if (i >= lag) rc = finish(i - lag);
        for (uint32_t j = i + 1 >= lag ? i + 1 - lag : 0; rc == NMZ_OK && i + 1 == n_traces && j <= i; ++j)
            if (plans[j]) rc = finish(j);
    }
    // on an error: every plan still alive waits for its work and goes
    for (auto *p : plans)
        if (p) plan_destroy_locked(p);
    seeds_destroy_locked(ss);
    return rc;
}

int nmz_replayable_sweep_seeds_topk_dev(nmz_replayable_plan *plan, const nmz_replayable_seeds *seeds, uint64_t seed0,
                                        uint32_t k, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk, void *stream) {
    NMZ_CHECK(plan != nullptr && seeds != nullptr, "NULL argument");
    NMZ_CHECK(seeds->ctx->device == plan->ctx->device, "the seed set and the plan are on different devices");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = stream ? (hipStream_t)stream : plan->ctx->stream;
    return replayable_run(plan, st, nullptr, nullptr, seeds->S, d_stats, seed0, k, d_topk, 0, seeds);
}

int nmz_replayable_sweep_decimal_topk_dev(nmz_replayable_plan *plan, uint64_t seed_lo, uint64_t n_seeds, uint32_t k,
                                          nmz_sched_stats *d_stats, nmz_topk_entry *d_topk, void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    NMZ_CHECK(n_seeds < (1ULL << 32), "at most 2^32-1 seeds per call");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = stream ? (hipStream_t)stream : plan->ctx->stream;
    return replayable_run(plan, st, nullptr, nullptr, n_seeds, d_stats, seed_lo, k, d_topk, seed_lo);
}

int nmz_replayable_sweep(nmz_ctx *ctx, const uint32_t *seed_off, const uint8_t *seed_bytes, uint64_t n_seeds,
                         const uint32_t *hint_off, const uint8_t *hint_bytes, uint32_t n_events,
                         int64_t max_interval_ns, nmz_sched_stats *stats, int64_t *delays,
                         uint64_t n_dump_seeds, uint32_t k, nmz_topk_entry *topk) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_seeds == 0 || seed_off, "seed_off is NULL");
    NMZ_CHECK(n_dump_seeds <= n_seeds, "n_dump_seeds > n_seeds");
    NMZ_CHECK(n_seeds < (1ULL << 32), "at most 2^32-1 seeds per call");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = ctx->stream;
    nmz_replayable_plan *plan = nullptr;
    NMZ_TRY(plan_create(ctx, hint_off, hint_bytes, n_events, max_interval_ns, n_seeds, &plan));
    struct PlanGuard {
        nmz_replayable_plan *p;
        ~PlanGuard() {
            plan_wait_uses(p);  // pooled buffers: no work may still use them
            p->plan_mem.release();
            p->seed_scratch.release();
            p->partial.release();
            p->topk_lists.release();
            p->oq_mem.release();
            p->wt.mem.release();
            p->wt.aux.release();
            p->wt_topk.release();
            delete p;
        }
    } pg{plan};

    const uint64_t sbytes = n_seeds ? seed_off[n_seeds] : 0;
    const uint64_t tk_entries = topk_scratch_entries(n_seeds, k);
    size_t need = Carve::bytes_for(n_seeds + 1, 4) + Carve::bytes_for(sbytes + 1, 1) +
                  Carve::bytes_for(n_seeds + 1, sizeof(nmz_sched_stats)) +
                  Carve::bytes_for(n_dump_seeds * n_events + 1, 8) + Carve::bytes_for(tk_entries + k + 1, 24);
    NMZ_TRY(ctx->buf[0].ensure(need));
    Carve cv(ctx->buf[0].ptr);
    uint32_t *d_soff = cv.take<uint32_t>(n_seeds + 1);
    uint8_t *d_sb = cv.take<uint8_t>(sbytes + 1);
    nmz_sched_stats *d_stats = cv.take<nmz_sched_stats>(n_seeds + 1);
    int64_t *d_dump = cv.take<int64_t>(n_dump_seeds * n_events + 1);
    nmz_topk_entry *d_tk = cv.take<nmz_topk_entry>(tk_entries + k + 1);
    if (n_seeds) {
        NMZ_HIP(hipMemcpyAsync(d_soff, seed_off, (n_seeds + 1) * 4, hipMemcpyHostToDevice, st));
        if (sbytes) NMZ_HIP(hipMemcpyAsync(d_sb, seed_bytes, sbytes, hipMemcpyHostToDevice, st));
    }
    NMZ_TRY(replayable_run(plan, st, d_soff, d_sb, n_seeds, d_stats));
    if (n_dump_seeds && n_events) {
        hipLaunchKernelGGL(k_replayable_dump, dim3(ceil_div(n_dump_seeds * n_events, 256)), dim3(256), 0, st, d_soff,
                           d_sb, n_dump_seeds, plan->d_hoff, plan->d_hbytes, n_events, plan->mod.m, d_dump);
        NMZ_HIP(hipGetLastError());
    }
    if (k) NMZ_TRY(topk_select(st, d_stats, n_seeds, 0, k, d_tk, d_tk + tk_entries));
    if (stats && n_seeds)
        NMZ_HIP(hipMemcpyAsync(stats, d_stats, n_seeds * sizeof(nmz_sched_stats), hipMemcpyDeviceToHost, st));
    if (delays && n_dump_seeds && n_events)
        NMZ_HIP(hipMemcpyAsync(delays, d_dump, n_dump_seeds * n_events * 8, hipMemcpyDeviceToHost, st));
    if (topk && k) NMZ_HIP(hipMemcpyAsync(topk, d_tk + tk_entries, k * sizeof(nmz_topk_entry), hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

// Online decisions on the calling host thread (Replayable.QueueEvent decides at enqueue, replayablepolicy.go:
// 116-126): FNV-1a 64 over seed || hint, then % uint64(maxInterval) -- k_replayable_dump's direct form.
int nmz_replayable_decide_host(const uint8_t *seed, uint32_t seed_len, const uint32_t *hint_off,
                               const uint8_t *hint_bytes, uint32_t n_events, int64_t max_interval_ns,
                               int64_t *delays) {
    if (n_events == 0) return NMZ_OK;
    NMZ_CHECK(hint_off && delays && (seed_len == 0 || seed), "NULL argument");
    const uint64_t m = (uint64_t)max_interval_ns;  // uint64(r.MaxInterval), replayablepolicy.go:110
    uint64_t h0 = FNV_OFFSET;
    for (uint32_t i = 0; i < seed_len; ++i) h0 = fnv_step(h0, seed[i]);
    for (uint32_t e = 0; e < n_events; ++e) {
        NMZ_CHECK(hint_off[e] <= hint_off[e + 1], "hint offsets must not decrease");
        NMZ_CHECK(hint_off[e] == hint_off[e + 1] || hint_bytes, "hint_bytes is NULL");
        if (m == 0) {  // :101-104
            delays[e] = 0;
            continue;
        }
        uint64_t h = h0;
        for (uint32_t b = hint_off[e]; b < hint_off[e + 1]; ++b) h = fnv_step(h, hint_bytes[b]);
        delays[e] = (int64_t)(h % m);
    }
    return NMZ_OK;
}

// Online decisions for one seed (Replayable.QueueEvent -> determineInterval, replayablepolicy.go:100-126): a batch
// of n pending events, one thread per event (k_replayable_dump: plain FNV over seed || hint, then % m). No plan:
// a batch of a few events needs no correction tables, only the launch.
int nmz_replayable_decide(nmz_ctx *ctx, const uint8_t *seed, uint32_t seed_len, const uint32_t *hint_off,
                          const uint8_t *hint_bytes, uint32_t n_events, int64_t max_interval_ns, int64_t *delays) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_events == 0) return NMZ_OK;
    NMZ_CHECK(hint_off && delays && (seed_len == 0 || seed), "NULL argument");
    if (max_interval_ns == 0) {  // :101-104
        for (uint32_t e = 0; e < n_events; ++e) delays[e] = 0;
        return NMZ_OK;
    }
    for (uint32_t e = 0; e < n_events; ++e) NMZ_CHECK(hint_off[e] <= hint_off[e + 1], "hint offsets must not decrease");
    const uint32_t hbytes = hint_off[n_events];
    NMZ_CHECK(hbytes == 0 || hint_bytes, "hint_bytes is NULL");
    hipStream_t st = ctx->stream;
    NMZ_TRY(ctx->buf[8].ensure(Carve::bytes_for(2, 4) + Carve::bytes_for(seed_len + 1, 1) +
                               Carve::bytes_for(n_events + 1, 4) + Carve::bytes_for(hbytes + 1, 1) +
                               Carve::bytes_for(n_events, 8) + 256));
    Carve cv(ctx->buf[8].ptr);
    uint32_t *d_soff = cv.take<uint32_t>(2);
    uint8_t *d_sb = cv.take<uint8_t>(seed_len + 1);
    uint32_t *d_hoff = cv.take<uint32_t>(n_events + 1);
    uint8_t *d_hb = cv.take<uint8_t>(hbytes + 1);
    int64_t *d_out = cv.take<int64_t>(n_events);
    const uint32_t soff[2] = {0, seed_len};
    NMZ_HIP(hipMemcpyAsync(d_soff, soff, 8, hipMemcpyHostToDevice, st));
    if (seed_len) NMZ_HIP(hipMemcpyAsync(d_sb, seed, seed_len, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_hoff, hint_off, (n_events + 1) * 4, hipMemcpyHostToDevice, st));
    if (hbytes) NMZ_HIP(hipMemcpyAsync(d_hb, hint_bytes, hbytes, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_replayable_dump, dim3(ceil_div(n_events, 256)), dim3(256), 0, st, d_soff, d_sb, (uint64_t)1,
                       d_hoff, d_hb, n_events, (uint64_t)max_interval_ns, d_out);
    NMZ_HIP(hipGetLastError());
    NMZ_HIP(hipMemcpyAsync(delays, d_out, (uint64_t)n_events * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

}  // extern "C"
