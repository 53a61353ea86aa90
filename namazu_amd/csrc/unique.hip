// Trace equality classes on the GPU: the `nmz tools visualize` unique-trace count
// (cli/tools/visualize.go:51-172), exact and partial-order reduced.
//
//   exact (seenBefore, :51-60):  SingleTrace.Equals, element-wise equality of the
//       action sequence (util/signal/misc.go:22-35).
//   partial order (seenBeforePOR / tracesEqualInPO, :62-136): each trace is projected
//       per entity (createTracesPerEntity: the events of its actions grouped by
//       EntityID(), in trace order, actions without an event skipped); two traces
//       are equal iff they hold the same entities and, per entity, element-wise
//       equal event sequences (Event.Equals).
//
// Both are equivalence relations, and the reference's loop keeps a trace iff no
// earlier trace equals it, so trace i is a repeat iff some j < i is equal to it.
//
// Signature: a trace is the multiset {(s_e, r_e)} of its symbols with their rank:
// the position for exact mode, the index among the same entity's elements for PO
// mode. The event symbol already holds the entity (the event JSON carries it), so
// for PO mode the multiset determines every per-entity sequence and vice versa.
// A multiset is hashed by summing a 64-bit mix of each pair mod 2^64 (an additive
// multiset hash, Clarke et al. 2003) under two different mixes, plus the element
// count: 128 bits per trace, order independent, so lanes can add in any order.
// The rank's part of each mix comes from a per-context table (65,536 ranks).
// Equal traces always give equal signatures; distinct ones collide with
// probability ~2^-128 per pair (the symbols themselves are 64-bit FNV event
// hashes).
//
// k_trace_sig: one wave per trace, 64 elements per step. PO ranks come from
// per-wave LDS counters indexed by the element's entity id (dense per trace,
// assigned by the host while it reads the trace): the lanes of one entity within
// a step are the intersection of one ballot per bit of the id (ceil(log2 ids)
// ballots), rank = counter + number of lower lanes in that set. Classes: radix sort of (sig hi, sig lo) with the
// trace index as payload (stable, so equal signatures keep index order), then
// first_equal[i] = the index at the start of i's run (max-scan of run heads).
#include <hipcub/hipcub.hpp>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

constexpr uint32_t SIG_WAVES = 4;             // waves (traces) per workgroup
constexpr uint32_t SIG_MAX_ENT_LDS = 4096;    // entity counters per wave at 4 waves per workgroup (64 KiB)
constexpr uint32_t SIG_MAX_ENT = 16384;       // one wave per workgroup beyond that
constexpr uint32_t SIG_MASK_ENT = 1024;       // entity masks (k_trace_sig MODE 2) up to this many entities: 48 KiB
#ifndef NMZ_SIG_U
#define NMZ_SIG_U 4
#endif
constexpr uint32_t SIG_U = NMZ_SIG_U;  // 64-element steps loaded together per wave
#ifndef NMZ_SIG_PIPE
#define NMZ_SIG_PIPE 2
#endif
#ifndef NMZ_SIG_UX
#define NMZ_SIG_UX 4
#endif
constexpr int SIG_PIPE = NMZ_SIG_PIPE;  // PO modes: the rank-key gather mixed one step later (1) or after the
                                       // batch's ranks (2) (k_trace_sig)

__device__ __forceinline__ uint64_t fmix64(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    x *= 0xc4ceb9fe1a85ec53ULL;
    x ^= x >> 33;
    return x;
}

// per-rank keys: RANK_KEYS ranks in a table (computed once per context), larger ranks inline
constexpr uint32_t RANK_KEYS = 65536;

__device__ __forceinline__ uint64_t rank_key_a(uint32_t r) { return fmix64((uint64_t)r + 0x9e3779b97f4a7c15ULL); }
__device__ __forceinline__ uint64_t rank_key_b(uint32_t r) {
    return fmix64(((uint64_t)r << 32 | (r ^ 0x5bd1e995u)) + 0x632be59bd9b4e019ULL);
}

__global__ void k_rank_keys(ulonglong2 *__restrict__ keys) {
    const uint32_t r = blockIdx.x * blockDim.x + threadIdx.x;
    if (r < RANK_KEYS) keys[r] = make_ulonglong2(rank_key_a(r), rank_key_b(r));
}

// the pair (symbol s, rank r) -> two 64-bit summands: t = fmix64(s ^ ka(r)) and a second, different nonlinear
// function of t and kb(r) (one more 64-bit multiply instead of another fmix64)
__device__ __forceinline__ ulonglong2 rank_keys(uint32_t r, const ulonglong2 *__restrict__ keys) {
    return r < RANK_KEYS ? keys[r] : make_ulonglong2(rank_key_a(r), rank_key_b(r));
}

__device__ __forceinline__ void mix2k(uint64_t s, ulonglong2 k, uint64_t &a, uint64_t &b) {
    const uint64_t t = fmix64(s ^ k.x);
    a = t;
    const uint64_t u = (t ^ k.y) * 0x94d049bb133111ebULL;
    b = u ^ (u >> 29);
}

__device__ __forceinline__ void mix2(uint64_t s, uint32_t r, const ulonglong2 *__restrict__ keys, uint64_t &a,
                                     uint64_t &b) {
    mix2k(s, rank_keys(r, keys), a, b);
}

// MODE 0: exact (rank = position); 1: PO, a lane's entity group from kbits ballots (one per bit of the id);
// 2: PO, the group from a per-wave LDS mask per entity (every lane ORs its bit into its entity's mask and reads it
// back: 2 LDS instructions instead of ~7 VALU per id bit; for traces of at most SIG_MASK_ENT entities)
template <int MODE>
__global__ __launch_bounds__(256) void k_trace_sig(const uint64_t *__restrict__ off, const uint64_t *__restrict__ sym,
                                                   const uint32_t *__restrict__ ent, uint32_t N, uint32_t max_ent,
                                                   uint32_t kbits, uint32_t waves_per_block,
                                                   const ulonglong2 *__restrict__ keys, uint64_t *__restrict__ sig) {
    constexpr bool PO = MODE != 0;
    extern __shared__ uint64_t sig_lds[];
    const uint32_t wv = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const uint32_t t = blockIdx.x * waves_per_block + wv;
    if (wv >= waves_per_block || t >= N) return;  // whole waves only: no block-wide barrier below
    // the wave's own counters (and entity masks, MODE 2) (LDS ops of one wave execute in order; compiler barriers
    // keep the order in the code)
    // MODE 2: every wave's [max_ent] u64 masks, then every wave's counters
    uint64_t *msk = sig_lds + (size_t)wv * max_ent;
    uint32_t *cnt = reinterpret_cast<uint32_t *>(MODE == 2 ? sig_lds + (size_t)waves_per_block * max_ent : sig_lds) +
                    (size_t)wv * max_ent;
    if (PO)
        for (uint32_t i = lane; i < max_ent; i += 64) {
            cnt[i] = 0;
            if (MODE == 2) msk[i] = 0;
        }
    __asm__ volatile("" ::: "memory");
    const uint64_t base = off[t], n = off[t + 1] - base;
    uint64_t acc1 = 0, acc2 = 0;
    uint32_t counted = 0;
    const uint64_t below = (1ULL << lane) - 1;
    bool pend = false;  // SIG_PIPE: the previous step's element, its keys gathered, not yet mixed
    uint64_t ps = 0;
    ulonglong2 pk = make_ulonglong2(0ull, 0ull);
    // PO mode: SIG_U steps' loads in flight per wave (one step at a time, the rank step's LDS round trip and the
    // next load's latency did not overlap: 0.73 -> 0.65 ms for 100k x 2,048); exact mode one step (measured
    // 3 % slower with four)
    constexpr uint32_t U = PO ? SIG_U : NMZ_SIG_UX;
    for (uint64_t c0 = 0; c0 < n; c0 += 64 * U) {
      uint64_t sv[U];
      uint32_t ev[U];
      ulonglong2 bk[U];  // SIG_PIPE 2: the batch's gathered keys, symbols and takes
      uint64_t bs[U];
      bool bt[U];
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) bt[k] = false;
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) {
          const uint64_t ic = min(c0 + 64 * k + lane, n - 1);  // n > 0 here: a valid element
          sv[k] = sym[base + ic];
          if (PO) ev[k] = ent[base + ic];
      }
#pragma unroll
      for (uint32_t k = 0; k < U; ++k) {
        const uint64_t c = c0 + 64 * k;
        if (c >= n) break;  // wave-uniform
        const uint64_t i = c + lane;
        const bool valid = i < n;
        const uint64_t s = valid ? sv[k] : 0;
        uint32_t rank = (uint32_t)i;
        bool take = valid;
        if (PO) {
            const uint32_t e0 = valid ? ev[k] : NMZ_NONE;
            take = valid && e0 < max_ent;  // NMZ_NONE (no event) skipped; ids past the bound never index LDS
            const uint32_t e = take ? e0 : 0u;
            if constexpr (MODE == 2) {
                // lanes holding the same entity: each ORs its bit into the entity's mask, then reads it back
                if (take) atomicOr(reinterpret_cast<unsigned long long *>(msk + e), 1ull << lane);
                __asm__ volatile("" ::: "memory");
                if (take) {
                    const uint64_t same = msk[e];
                    const uint32_t before = cnt[e];
                    rank = before + (uint32_t)__popcll(same & below);
                    // every lane of the wave has read (one LDS instruction each) before the group's last lane
                    // stores the count and clears the mask for the next step
                    __asm__ volatile("" ::: "memory");
                    if ((same >> lane) == 1ull) {
                        cnt[e] = before + (uint32_t)__popcll(same);
                        msk[e] = 0;
                    }
                }
            } else {
            // lanes holding the same entity: intersect, bit by bit of the id, the ballot of lanes that agree
            // on that bit (kbits ballots per 64 elements instead of one per distinct entity)
            // (as the lanes that differ from this one in some bit: one XOR-OR per ballot, no per-lane select)
            uint64_t diff = ~__builtin_amdgcn_ballot_w64(take);
            const uint32_t et = take ? e : 0xffffffffu;  // untaken lanes set every bit: no ballot needs `take`
            for (uint32_t b = 0; b < kbits; ++b) {
                const uint32_t bm = (uint32_t)((int32_t)(et << (31 - b)) >> 31);  // all ones when bit b is set
                const uint64_t B = __builtin_amdgcn_ballot_w64(bm != 0);
                diff |= B ^ (((uint64_t)bm << 32) | bm);
            }
            const uint64_t same = ~diff;
            if (take) {
                const uint32_t before = cnt[e];
                rank = before + (uint32_t)__popcll(same & below);
                // every lane of the wave has read (one LDS instruction) before the group's last lane stores
                __asm__ volatile("" ::: "memory");
                if ((same >> lane) == 1ull) cnt[e] = before + (uint32_t)__popcll(same);
            }
            }
        }
        if (SIG_PIPE == 2) {
            // the batch's ranks first (every step's keys gather in flight), the mixes after the batch
            bk[k] = take ? rank_keys(rank, keys) : make_ulonglong2(0ull, 0ull);
            bs[k] = s;
            bt[k] = take;
        } else if (PO && SIG_PIPE) {
            // software pipeline: this step's keys[rank] gather is issued now and mixed one step later, so its
            // latency overlaps the next step's LDS round trips (the rank chain) instead of stalling the wave
            const ulonglong2 kk = take ? rank_keys(rank, keys) : make_ulonglong2(0ull, 0ull);
            if (pend) {
                uint64_t a, b;
                mix2k(ps, pk, a, b);
                acc1 += a;
                acc2 += b;
                counted += 1;
            }
            pend = take;
            ps = s;
            pk = kk;
        } else if (take) {
            uint64_t a, b;
            mix2(s, rank, keys, a, b);
            acc1 += a;
            acc2 += b;
            counted += 1;
        }
      }
      if (SIG_PIPE == 2) {
#pragma unroll
        for (uint32_t k = 0; k < U; ++k)
            if (bt[k]) {
                uint64_t a, b;
                mix2k(bs[k], bk[k], a, b);
                acc1 += a;
                acc2 += b;
                counted += 1;
            }
      }
    }
    if (PO && SIG_PIPE == 1 && pend) {
        uint64_t a, b;
        mix2k(ps, pk, a, b);
        acc1 += a;
        acc2 += b;
        counted += 1;
    }
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) {
        acc1 += __shfl_xor(acc1, o, 64);
        acc2 += __shfl_xor(acc2, o, 64);
        counted += __shfl_xor(counted, o, 64);
    }
    if (lane == 0) {
        sig[2 * (uint64_t)t] = acc1 + fmix64((uint64_t)counted + 1);
        sig[2 * (uint64_t)t + 1] = acc2 ^ fmix64(((uint64_t)counted << 1) | 1);
    }
}

__global__ void k_sig_split(const uint64_t *__restrict__ sig, uint32_t N, uint64_t *__restrict__ lo,
                            uint64_t *__restrict__ hi, uint32_t *__restrict__ idx) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) {
        lo[i] = sig[2 * (uint64_t)i];
        hi[i] = sig[2 * (uint64_t)i + 1];
        idx[i] = i;
    }
}

__global__ void k_gather_u64(const uint64_t *__restrict__ src, const uint32_t *__restrict__ idx, uint32_t N,
                             uint64_t *__restrict__ dst) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < N) dst[p] = src[idx[p]];
}

// heads of runs of equal (hi, lo) in sorted order: start[p] = p at a head, 0 elsewhere (max-scanned below)
__global__ void k_sig_heads(const uint64_t *__restrict__ lo, const uint64_t *__restrict__ hi_sorted,
                            const uint32_t *__restrict__ idx_sorted, uint32_t N, uint32_t *__restrict__ start) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p >= N) return;
    bool head = p == 0;
    if (!head) {
        // lo halves of sorted neighbours, read through their trace indices
        head = hi_sorted[p] != hi_sorted[p - 1] || lo[idx_sorted[p]] != lo[idx_sorted[p - 1]];
    }
    start[p] = head ? p : 0;
}

__global__ void k_sig_first(const uint32_t *__restrict__ idx_sorted, const uint32_t *__restrict__ start, uint32_t N,
                            uint32_t *__restrict__ first_equal) {
    const uint32_t p = blockIdx.x * blockDim.x + threadIdx.x;
    if (p < N) first_equal[idx_sorted[p]] = idx_sorted[start[p]];
}

static int sig_launch(nmz_ctx *ctx, const uint64_t *d_off, const uint64_t *d_sym, const uint32_t *d_ent, uint32_t N,
                      uint32_t max_ent, uint64_t *d_sig, hipStream_t st) {
    if (N == 0) return NMZ_OK;
    DevBuf &kb = ctx->buf[14];  // rank keys, built once per context
    if (!kb.ptr) {
        NMZ_TRY(kb.ensure((size_t)RANK_KEYS * sizeof(ulonglong2)));
        // on the context's stream, waited for once: later launches on any stream see the finished table
        hipLaunchKernelGGL(k_rank_keys, dim3(RANK_KEYS / 256), dim3(256), 0, ctx->stream, kb.as<ulonglong2>());
        NMZ_HIP(hipGetLastError());
        NMZ_HIP(hipStreamSynchronize(ctx->stream));
    }
    const ulonglong2 *keys = kb.as<ulonglong2>();
    if (!d_ent) {
        hipLaunchKernelGGL(k_trace_sig<0>, dim3(ceil_div(N, SIG_WAVES)), dim3(64 * SIG_WAVES), 0, st, d_off, d_sym,
                           nullptr, N, 0u, 0u, SIG_WAVES, keys, d_sig);
    } else {
        NMZ_CHECK(max_ent <= SIG_MAX_ENT, "more than 16384 distinct entities in one trace");
        const uint32_t me = max_ent ? max_ent : 1;
        const uint32_t wpb = me <= SIG_MAX_ENT_LDS ? SIG_WAVES : 1;
        uint32_t kbits = 0;
        while ((1u << kbits) < me) ++kbits;
        const char *ab = ab_env("NMZ_SIG_MASKS");  // (A/B: NMZ_SIG_MASKS=0 takes the ballots)
        if (me <= SIG_MASK_ENT && !(ab && ab[0] == '0'))
            hipLaunchKernelGGL(k_trace_sig<2>, dim3(ceil_div(N, SIG_WAVES)), dim3(64 * SIG_WAVES),
                               (size_t)SIG_WAVES * me * 12, st, d_off, d_sym, d_ent, N, me, kbits, SIG_WAVES, keys,
                               d_sig);
        else
            hipLaunchKernelGGL(k_trace_sig<1>, dim3(ceil_div(N, wpb)), dim3(64 * wpb), (size_t)wpb * me * 4, st, d_off,
                               d_sym, d_ent, N, me, kbits, wpb, keys, d_sig);
    }
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// equality classes from signatures: first_equal[i] = smallest j with sig_j == sig_i
static int classes_launch(nmz_ctx *ctx, const uint64_t *d_sig, uint32_t N, uint32_t *d_first, hipStream_t st) {
    if (N == 0) return NMZ_OK;
    size_t sort_bytes = 0, scan_bytes = 0;
    NMZ_HIP(hipcub::DeviceRadixSort::SortPairs(nullptr, sort_bytes, (uint64_t *)nullptr, (uint64_t *)nullptr,
                                               (uint32_t *)nullptr, (uint32_t *)nullptr, (int)N, 0, 64, st));
    NMZ_HIP(hipcub::DeviceScan::InclusiveScan(nullptr, scan_bytes, (uint32_t *)nullptr, (uint32_t *)nullptr,
                                              hipcub::Max(), (int)N, st));
    DevBuf &scr = ctx->buf[6];
    NMZ_TRY(scr.ensure(4 * Carve::bytes_for(N, 8) + 4 * Carve::bytes_for(N, 4) +
                       Carve::bytes_for(std::max(sort_bytes, scan_bytes) + 1, 1)));
    Carve cv(scr.ptr);
    uint64_t *lo = cv.take<uint64_t>(N), *hi = cv.take<uint64_t>(N);
    uint64_t *k1 = cv.take<uint64_t>(N), *k2 = cv.take<uint64_t>(N);
    uint32_t *idx = cv.take<uint32_t>(N), *v1 = cv.take<uint32_t>(N), *v2 = cv.take<uint32_t>(N);
    uint32_t *start = cv.take<uint32_t>(N);
    void *tmp = cv.take<char>(std::max(sort_bytes, scan_bytes) + 1);
    const unsigned g = ceil_div(N, 256);
    hipLaunchKernelGGL(k_sig_split, dim3(g), dim3(256), 0, st, d_sig, N, lo, hi, idx);
    NMZ_HIP(hipGetLastError());
    // LSD: by lo, then (stable) by hi -> order (hi, lo, index)
    size_t b = sort_bytes;
    NMZ_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, b, lo, k1, idx, v1, (int)N, 0, 64, st));
    // hi keys in lo-sorted order
    hipLaunchKernelGGL(k_gather_u64, dim3(g), dim3(256), 0, st, hi, v1, N, k2);
    NMZ_HIP(hipGetLastError());
    b = sort_bytes;
    NMZ_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, b, k2, hi, v1, v2, (int)N, 0, 64, st));
    // hi now holds the sorted hi keys, v2 the trace indices in (hi, lo, index) order
    hipLaunchKernelGGL(k_sig_heads, dim3(g), dim3(256), 0, st, lo, hi, v2, N, start);
    NMZ_HIP(hipGetLastError());
    b = scan_bytes;
    NMZ_HIP(hipcub::DeviceScan::InclusiveScan(tmp, b, start, start, hipcub::Max(), (int)N, st));
    hipLaunchKernelGGL(k_sig_first, dim3(g), dim3(256), 0, st, v2, start, N, d_first);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

// Sorted distinct values of d_sym[0..total) (the bit-parallel ED plan's alphabet, ed.hip). A store holds
// ~10^8 event hashes over at most a few thousand distinct events, so the distinct set comes from hashing, not
// from sorting the store: each workgroup dedups its grid-stride share in an LDS open-addressing table (a plain
// read finds a present key, a 64-bit LDS compare-and-swap claims a free slot) and then inserts its distinct keys
// into one global table; a compaction writes the set out and a radix sort of those few keys orders it. The global
// table has far more slots than any set the plan accepts (cap < 2^16 distinct, 2^20 slots) and a probe sequence
// is bounded by the table size, so every insert ends even when the store has millions of distinct values: the
// count then passes cap and the caller takes its other path.
constexpr uint32_t DS_LDS_SLOTS = 4096, DS_LDS_MAX = 2048;  // per workgroup (32 KB); fill bound before going global
constexpr uint32_t DS_G_SLOTS = 1u << 20;                  // global table (8 MB)
constexpr uint64_t DS_EMPTY = ~0ull;                       // a free slot; the value itself is flagged separately

__device__ __forceinline__ uint32_t ds_hash(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdull;
    x ^= x >> 33;
    return (uint32_t)x;
}

// flags[0] = global distinct count, flags[1] = DS_EMPTY seen
__device__ __forceinline__ void ds_global_insert(unsigned long long *tab, uint32_t *flags, uint32_t cap, uint64_t x) {
    uint32_t h = ds_hash(x) & (DS_G_SLOTS - 1);
    for (uint32_t probe = 0; probe < DS_G_SLOTS; ++probe, h = (h + 1) & (DS_G_SLOTS - 1)) {
        const uint64_t cur = __hip_atomic_load(&tab[h], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (cur == x) return;
        if (cur != DS_EMPTY) continue;
        if (__hip_atomic_load(&flags[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) > cap) return;  // too many: stop
        const uint64_t old = atomicCAS(&tab[h], (unsigned long long)DS_EMPTY, (unsigned long long)x);
        if (old == DS_EMPTY) {
            atomicAdd(&flags[0], 1u);
            return;
        }
        if (old == x) return;
    }
    atomicMax(&flags[0], cap + 1);  // table exhausted (only with far more than cap distinct values)
}

__global__ __launch_bounds__(256) void k_distinct_insert(const uint64_t *__restrict__ sym, uint64_t total,
                                                         unsigned long long *__restrict__ tab, uint32_t *flags,
                                                         uint32_t cap) {
    __shared__ unsigned long long lt[DS_LDS_SLOTS];
    __shared__ uint32_t lcount;
    for (uint32_t i = threadIdx.x; i < DS_LDS_SLOTS; i += 256) lt[i] = DS_EMPTY;
    if (threadIdx.x == 0) lcount = 0;
    __syncthreads();
    bool saw_empty = false;
    const uint64_t stride = (uint64_t)gridDim.x * 256;
    for (uint64_t t = (uint64_t)blockIdx.x * 256 + threadIdx.x; t < total; t += stride) {
        const uint64_t x = sym[t];
        if (x == DS_EMPTY) {
            saw_empty = true;
            continue;
        }
        uint32_t h = ds_hash(x) & (DS_LDS_SLOTS - 1);
        bool done = false;
        for (uint32_t probe = 0; probe < DS_LDS_SLOTS && !done; ++probe, h = (h + 1) & (DS_LDS_SLOTS - 1)) {
            const uint64_t cur = lt[h];
            if (cur == x) {
                done = true;
            } else if (cur == DS_EMPTY) {
                if (atomicAdd(&lcount, 0u) >= DS_LDS_MAX) break;  // this workgroup's table is full enough: global
                const uint64_t old = atomicCAS(&lt[h], (unsigned long long)DS_EMPTY, (unsigned long long)x);
                if (old == DS_EMPTY) {
                    atomicAdd(&lcount, 1u);
                    done = true;
                } else if (old == x) {
                    done = true;
                }
            }
        }
        if (!done) ds_global_insert(tab, flags, cap, x);
    }
    if (saw_empty) flags[1] = 1u;
    __syncthreads();
    for (uint32_t i = threadIdx.x; i < DS_LDS_SLOTS; i += 256)
        if (lt[i] != DS_EMPTY) ds_global_insert(tab, flags, cap, lt[i]);
}

__global__ __launch_bounds__(256) void k_distinct_compact(const unsigned long long *__restrict__ tab, uint32_t *flags,
                                                          uint32_t cap, uint64_t *__restrict__ out) {
    const uint32_t i = blockIdx.x * 256 + threadIdx.x;
    if (i >= DS_G_SLOTS) return;
    const uint64_t x = tab[i];
    if (x == DS_EMPTY) return;
    const uint32_t at = atomicAdd(&flags[2], 1u);
    if (at < cap) out[at] = x;
}

// d_uniq: capacity cap + 1; *n_uniq > cap when there are more than cap distinct values (d_uniq is then not filled)
int device_unique_u64(const uint64_t *d_sym, uint64_t total, uint64_t *d_uniq, uint64_t cap, uint64_t *n_uniq,
                      hipStream_t st) {
    *n_uniq = 0;
    if (total == 0) return NMZ_OK;
    NMZ_CHECK(cap > 0 && cap < DS_G_SLOTS / 8, "internal: distinct-set capacity out of range");
    const uint32_t c32 = (uint32_t)cap;
    size_t sort_bytes = 0;
    NMZ_HIP(hipcub::DeviceRadixSort::SortKeys(nullptr, sort_bytes, (const uint64_t *)nullptr, (uint64_t *)nullptr,
                                              (int)cap + 1, 0, 64, st));
    DevBuf scr;
    NMZ_TRY(scr.ensure(Carve::bytes_for(DS_G_SLOTS, 8) + Carve::bytes_for(4, 4) + Carve::bytes_for(cap + 1, 8) +
                       Carve::bytes_for(sort_bytes + 1, 1)));
    Carve cv(scr.ptr);
    unsigned long long *tab = cv.take<unsigned long long>(DS_G_SLOTS);
    uint32_t *flags = cv.take<uint32_t>(4);
    uint64_t *raw = cv.take<uint64_t>(cap + 1);
    void *tmp = cv.take<char>(sort_bytes + 1);
    int rc = NMZ_OK;
    uint32_t hf[4] = {0, 0, 0, 0};
    auto ok = [&](hipError_t e) {
        if (e != hipSuccess) rc = NMZ_EHIP;
        return rc == NMZ_OK;
    };
    const uint32_t blocks = (uint32_t)std::min<uint64_t>(2048, (total + 255) / 256);
    if (ok(hipMemsetAsync(tab, 0xff, (size_t)DS_G_SLOTS * 8, st)) && ok(hipMemsetAsync(flags, 0, 16, st))) {
        hipLaunchKernelGGL(k_distinct_insert, dim3(blocks), dim3(256), 0, st, d_sym, total, tab, flags, c32);
        hipLaunchKernelGGL(k_distinct_compact, dim3(DS_G_SLOTS / 256), dim3(256), 0, st, tab, flags, c32, raw);
        if (ok(hipGetLastError()) && ok(hipMemcpyAsync(hf, flags, 16, hipMemcpyDeviceToHost, st)))
            ok(hipStreamSynchronize(st));
    }
    if (rc == NMZ_OK) {
        const uint64_t n = (uint64_t)hf[2] + hf[1];
        if (hf[0] > c32 || n > cap) {
            *n_uniq = cap + 1;
        } else {
            size_t b = sort_bytes;
            if (hf[2] > 0) ok(hipcub::DeviceRadixSort::SortKeys(tmp, b, raw, d_uniq, (int)hf[2], 0, 64, st));
            const uint64_t top = DS_EMPTY;  // the largest value: last in sorted order
            if (rc == NMZ_OK && hf[1]) ok(hipMemcpyAsync(d_uniq + hf[2], &top, 8, hipMemcpyHostToDevice, st));
            if (rc == NMZ_OK) ok(hipStreamSynchronize(st));  // before the scratch goes back
            *n_uniq = n;
        }
    }
    scr.release();
    return rc == NMZ_OK ? NMZ_OK : fail(NMZ_EHIP, "device distinct-symbol set failed");
}

}  // namespace nmz

using namespace nmz;

extern "C" {

int nmz_trace_signatures(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint32_t *entity,
                         uint32_t n_traces, uint64_t *sig) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0) return NMZ_OK;
    NMZ_CHECK(off && sig, "NULL argument");
    const uint64_t total = off[n_traces];
    NMZ_CHECK(total == 0 || sym, "sym is NULL");
    uint32_t max_ent = 0;
    if (entity)
        for (uint64_t i = 0; i < total; ++i)
            if (entity[i] != NMZ_NONE) max_ent = std::max(max_ent, entity[i] + 1);
    hipStream_t st = ctx->stream;
    NMZ_TRY(ctx->buf[7].ensure(Carve::bytes_for(n_traces + 1, 8) + Carve::bytes_for(total + 1, 8) +
                               Carve::bytes_for(total + 1, 4) + Carve::bytes_for(2 * (uint64_t)n_traces, 8)));
    Carve cv(ctx->buf[7].ptr);
    uint64_t *d_off = cv.take<uint64_t>(n_traces + 1);
    uint64_t *d_sym = cv.take<uint64_t>(total + 1);
    uint32_t *d_ent = cv.take<uint32_t>(total + 1);
    uint64_t *d_sig = cv.take<uint64_t>(2 * (uint64_t)n_traces);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (n_traces + 1) * 8, hipMemcpyHostToDevice, st));
    if (total) NMZ_HIP(hipMemcpyAsync(d_sym, sym, total * 8, hipMemcpyHostToDevice, st));
    if (total && entity) NMZ_HIP(hipMemcpyAsync(d_ent, entity, total * 4, hipMemcpyHostToDevice, st));
    NMZ_TRY(sig_launch(ctx, d_off, d_sym, entity ? d_ent : nullptr, n_traces, max_ent, d_sig, st));
    NMZ_HIP(hipMemcpyAsync(sig, d_sig, 2 * (uint64_t)n_traces * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_unique_traces(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint32_t *entity,
                      uint32_t n_traces, uint32_t *first_equal) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0) return NMZ_OK;
    NMZ_CHECK(off && first_equal, "NULL argument");
    const uint64_t total = off[n_traces];
    NMZ_CHECK(total == 0 || sym, "sym is NULL");
    for (uint32_t i = 0; i < n_traces; ++i) NMZ_CHECK(off[i] <= off[i + 1], "offsets must be non-decreasing");
    uint32_t max_ent = 0;
    if (entity)
        for (uint64_t i = 0; i < total; ++i)
            if (entity[i] != NMZ_NONE) max_ent = std::max(max_ent, entity[i] + 1);
    hipStream_t st = ctx->stream;
    NMZ_TRY(ctx->buf[7].ensure(Carve::bytes_for(n_traces + 1, 8) + Carve::bytes_for(total + 1, 8) +
                               Carve::bytes_for(total + 1, 4) + Carve::bytes_for(2 * (uint64_t)n_traces, 8) +
                               Carve::bytes_for(n_traces, 4)));
    Carve cv(ctx->buf[7].ptr);
    uint64_t *d_off = cv.take<uint64_t>(n_traces + 1);
    uint64_t *d_sym = cv.take<uint64_t>(total + 1);
    uint32_t *d_ent = cv.take<uint32_t>(total + 1);
    uint64_t *d_sig = cv.take<uint64_t>(2 * (uint64_t)n_traces);
    uint32_t *d_first = cv.take<uint32_t>(n_traces);
    NMZ_HIP(hipMemcpyAsync(d_off, off, (n_traces + 1) * 8, hipMemcpyHostToDevice, st));
    if (total) NMZ_HIP(hipMemcpyAsync(d_sym, sym, total * 8, hipMemcpyHostToDevice, st));
    if (total && entity) NMZ_HIP(hipMemcpyAsync(d_ent, entity, total * 4, hipMemcpyHostToDevice, st));
    NMZ_TRY(sig_launch(ctx, d_off, d_sym, entity ? d_ent : nullptr, n_traces, max_ent, d_sig, st));
    {
        KernelTimer kt(ctx, st, "unique_classes");
        NMZ_TRY(classes_launch(ctx, d_sig, n_traces, d_first, st));
    }
    NMZ_HIP(hipMemcpyAsync(first_equal, d_first, (uint64_t)n_traces * 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    return NMZ_OK;
}

int nmz_unique_traces_dev(nmz_ctx *ctx, const uint64_t *d_off, const uint64_t *d_sym, const uint32_t *d_entity,
                          uint32_t n_traces, uint32_t max_entities, uint64_t *d_sig, uint32_t *d_first_equal,
                          void *stream) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_traces == 0) return NMZ_OK;
    NMZ_CHECK(d_off && d_sig && d_first_equal, "NULL argument");
    hipStream_t st = stream ? (hipStream_t)stream : ctx->stream;
    {
        KernelTimer kt(ctx, st, "trace_sig");
        NMZ_TRY(sig_launch(ctx, d_off, d_sym, d_entity, n_traces, max_entities, d_sig, st));
    }
    return classes_launch(ctx, d_sig, n_traces, d_first_equal, st);
}

}  // extern "C"
