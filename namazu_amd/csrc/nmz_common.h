// Shared host/device definitions for libnmz_gpu.so (gfx950 only).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <map>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/nmz_gpu.h"

// ---------------------------------------------------------------------------
// error plumbing (thread-local message, int status codes of nmz_gpu.h)
// ---------------------------------------------------------------------------
namespace nmz {

void set_error(const std::string &msg);
int fail(int code, const std::string &msg);

#define NMZ_HIP(call)                                                                   \
    do {                                                                                \
        hipError_t e_ = (call);                                                         \
        if (e_ != hipSuccess)                                                           \
            return ::nmz::fail(NMZ_EHIP, std::string(#call) + ": " + hipGetErrorString(e_)); \
    } while (0)

#define NMZ_CHECK(cond, msg)                                                            \
    do {                                                                                \
        if (!(cond)) return ::nmz::fail(NMZ_EINVAL, (msg));                             \
    } while (0)

#define NMZ_TRY(expr)                                                                   \
    do {                                                                                \
        int rc_ = (expr);                                                               \
        if (rc_ != NMZ_OK) return rc_;                                                  \
    } while (0)

// Grow-only device scratch buffer owned by a context. With a pool (a plan's buffers: the context's list of
// free buffers), release() hands the memory back to the pool and ensure() reuses a pooled buffer before it
// allocates, so creating and destroying plans does not hipMalloc / hipFree (hipFree synchronises the device).
struct DevBuf {
    void *ptr = nullptr;
    size_t cap = 0;
    std::vector<DevBuf> *pool = nullptr;
    uint64_t gen = 0;  // bumped whenever ensure() hands out a different allocation (its contents are then undefined)
    int ensure(size_t bytes);
    void release();
    template <typename T>
    T *as() const { return static_cast<T *>(ptr); }
};

// Grow-only pinned host staging owned by a context: a plan's inputs are packed here and reach the device in one
// asynchronous copy (a pageable hipMemcpyAsync stages through a driver buffer and returns only when that is done).
// The copy reading it is marked with an event (mark); ensure() waits for it before the buffer is packed again,
// so a build that returns before its upload finished (nmz_replayable_plan_create_async) is safe.
struct HostPin {
    void *ptr = nullptr;
    size_t cap = 0;
    hipEvent_t busy = nullptr;  // recorded after the last copy out of the buffer
    int ensure(size_t bytes);   // waits for that copy, then grows (a power of two of at least 1 MiB)
    int mark(hipStream_t st);
    void release();
};

}  // namespace nmz

// Optional HIP-event timing of the dominant kernels (bench.py reads it).
struct NmzTiming {
    bool enabled = false;
    bool spans_only = false;  // NMZ_TIMING_SPANS: span slots, no events
    std::map<std::string, std::vector<std::pair<hipEvent_t, hipEvent_t>>> events;
    std::vector<hipEvent_t> pool;
    // in-kernel execution spans: slot = {max ~start, max end} of wall_clock64() over the launch's workgroups
    unsigned long long *span_dev = nullptr;
    uint32_t span_next = 0;
    std::map<std::string, std::vector<uint32_t>> spans;
};
constexpr uint32_t NMZ_SPAN_SLOTS = 4096;

struct nmz_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    std::mutex mu;
    int n_cu = 0;
    // scratch slots reused across calls (host-pointer entry points)
    nmz::DevBuf buf[16];
    std::vector<nmz::DevBuf> pool;  // free plan buffers (DevBuf::pool), freed by nmz_close
    nmz::HostPin pin[2];             // pinned staging of plan inputs ([0] replayable plan, [1] its wavelet classes)
    bool wt_lds_attr = false;        // the wavelet-tree kernels' LDS attribute is set on this context's device
    // nmz_replayable_sweep_traces: a private second context (the other half of the plan builds), two sweep streams
    // with an event each, and pinned staging for the top-k lists; created on first use
    nmz_ctx *helper = nullptr;
    hipStream_t sweep_st[2] = {nullptr, nullptr};
    hipEvent_t sweep_ev[3] = {nullptr, nullptr, nullptr};
    nmz::HostPin tkpin;
    NmzTiming timing;
};

namespace nmz {

// Records start/stop events around a kernel launch when timing is enabled.
struct KernelTimer {
    nmz_ctx *ctx;
    hipStream_t st;
    const char *name;
    hipEvent_t a = nullptr, b = nullptr;
    bool spans_only = false;
    KernelTimer(nmz_ctx *c, hipStream_t s, const char *n);
    ~KernelTimer();
    // a fresh span slot for a kernel that records its own execution span (nullptr when timing is off)
    unsigned long long *span();
};

// RAII: the caller's current HIP device is restored on return, so a call never changes the device of the thread
// that made it (torch or other HIP work on that thread keeps its own).
struct DeviceRestore {
    int prev = -1;
    DeviceRestore() {
        if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    }
    ~DeviceRestore() {
        int cur = -1;
        if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
    }
};

// RAII: bind the calling OS thread to the context's device for the call (cgo threads migrate), then restore the
// caller's device.
struct CtxGuard {
    std::lock_guard<std::mutex> lk;
    DeviceRestore restore;
    int rc = NMZ_OK;
    explicit CtxGuard(nmz_ctx *c) : lk(c->mu) {
        if (hipSetDevice(c->device) != hipSuccess) rc = fail(NMZ_EHIP, "hipSetDevice failed");
    }
};

// ---------------------------------------------------------------------------
// FNV-1a 64 (Go hash/fnv New64a) and the low-byte decomposition used by the
// sweep kernels:  F_hint(h) = h * P^len + C_hint[h & 0xff]   (mod 2^64)
// The low byte of the FNV state evolves independently of the high bits
// (x * P mod 256 only sees x mod 256), so every XOR a hint byte applies is an
// additive offset that depends only on h & 0xff.
// ---------------------------------------------------------------------------
constexpr uint64_t FNV_OFFSET = 0xcbf29ce484222325ULL;
constexpr uint64_t FNV_PRIME = 0x100000001b3ULL;

__host__ __device__ inline uint64_t fnv_step(uint64_t h, uint32_t b) {
    return (h ^ (uint64_t)b) * FNV_PRIME;
}

__host__ __device__ inline uint64_t fnv_pow(uint32_t n) {
    uint64_t r = 1, b = FNV_PRIME;
    while (n) {
        if (n & 1) r *= b;
        b *= b;
        n >>= 1;
    }
    return r;
}

// ---------------------------------------------------------------------------
// u64 modulus by a launch constant m.
//   FAST   : 0 < m < 2^30, used through the carry decomposition (see replayable.hip)
//   GENERAL: any m > 0 (u64 remainder)
// ---------------------------------------------------------------------------
enum ModKind : int { MOD_ZERO = 0, MOD_FAST = 1, MOD_GENERAL = 2 };

struct ModParams {
    uint64_t m;
    uint32_t m32;
    uint32_t k64;   // 2^64 mod m (m < 2^32)
    uint32_t m_k64; // (m - k64) mod m, added when the 64-bit add carried (m < 2^32)
    uint64_t mu;    // floor(2^64 / m) for mod_barrett_small / mod_barrett64 (m < 2^32; 2^64 - 1 for m = 1)
    int kind;
    bool m32ok;     // 0 < m < 2^32: residues fit 32 bits (the order-query statistics apply)
};

inline ModParams make_mod(uint64_t m) {
    ModParams p{};
    p.m = m;
    p.m32ok = m != 0 && m < (1ULL << 32);
    if (p.m32ok) {
        p.m32 = (uint32_t)m;
        uint64_t k = (uint64_t)(((unsigned __int128)1 << 64) % m);
        p.k64 = (uint32_t)k;
        p.m_k64 = (uint32_t)((m - k) % m);
        p.mu = m == 1 ? ~0ULL : (uint64_t)(((unsigned __int128)1 << 64) / m);
    }
    p.kind = m == 0 ? MOD_ZERO : (m < (1ULL << 30) ? MOD_FAST : MOD_GENERAL);
    return p;
}

// v mod m for any 64-bit v and m < 2^31, mu = floor(2^64 / m) (2^64 - 1 for m = 1): q = floor(v * mu / 2^64)
// is floor(v / m) or one less, so r = v - q*m < 2m < 2^32 and only the low words are needed:
// r = v_lo - q_lo * m (mod 2^32), with v*mu = vl*mul + (vh*mul + vl*muh) 2^32 + vh*muh 2^64.
// high word of a 32 x 32-bit product (v_mul_hi_u32 on the device; the host decision path shares the code)
__host__ __device__ __forceinline__ uint32_t umulhi32(uint32_t a, uint32_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umulhi(a, b);
#else
    return (uint32_t)(((uint64_t)a * b) >> 32);
#endif
}
__host__ __device__ __forceinline__ uint64_t umulhi64(uint64_t a, uint64_t b) {
#ifdef __HIP_DEVICE_COMPILE__
    return __umul64hi(a, b);
#else
    return (uint64_t)(((unsigned __int128)a * b) >> 64);
#endif
}

__host__ __device__ __forceinline__ uint32_t mod_barrett_small(uint64_t v, uint32_t m, uint64_t mu) {
    const uint32_t vl = (uint32_t)v, vh = (uint32_t)(v >> 32);
    const uint32_t mul = (uint32_t)mu, muh = (uint32_t)(mu >> 32);
    const uint64_t a = (uint64_t)vh * mul + umulhi32(vl, mul);
    const uint64_t b = (uint64_t)vl * muh + (uint32_t)a;
    const uint32_t ql = vh * muh + (uint32_t)(a >> 32) + (uint32_t)(b >> 32);
    const uint32_t r = vl - ql * m;
    uint32_t t;
    return __builtin_sub_overflow(r, m, &t) ? r : t;
}

// v mod m for any 64-bit v and 0 < m < 2^32, mu = floor(2^64 / m): the quotient estimate is floor(v / m) or one
// less, so one conditional subtract.
__host__ __device__ __forceinline__ uint32_t mod_barrett64(uint64_t v, uint64_t m, uint64_t mu) {
    const uint64_t r = v - umulhi64(v, mu) * m;
    return (uint32_t)(r >= m ? r - m : r);
}

// Reduce s in [0, 3m) to [0, m) for m < 2^30 with two branch-free min steps.
__device__ inline uint32_t reduce3m(uint32_t s, uint32_t m) {
    s = min(s, s - m);
    return min(s, s - m);
}

// ---------------------------------------------------------------------------
// per-seed statistics accumulator
// ---------------------------------------------------------------------------
__host__ __device__ inline void stats_empty(nmz_sched_stats &s) {
    s.sum_delay_ns = 0;
    s.max_delay_ns = INT64_MIN;
    s.argmax_event = NMZ_NONE;
    s.n_fault = 0;
    s.first_fault = NMZ_NONE;
    s.flags = 0;
}

// ---------------------------------------------------------------------------
// launch helpers
// ---------------------------------------------------------------------------
inline unsigned ceil_div(uint64_t a, uint64_t b) { return (unsigned)((a + b - 1) / b); }

// seed bucketing by FNV low byte (shared by both sweeps): a counting sort with no global atomics. The prefix
// kernels hash blocks of BUCKET_BLK seeds and store each block's 256 bucket counts in its own row of b.hist (every
// row is written whole, so nothing needs zeroing); k_bucket_colscan turns each bucket's column of rows, in place,
// into the rows' offsets inside the bucket and the bucket's total; k_bucket_scatter scans the totals into the
// bucket starts and writes each block's seeds from start + row offset (block 0 also writes the starts and the work
// units). (Device-scope atomics on 256 shared counters from every block -- the previous form -- serialise on
// their words: ~11 ns each, 11 + 16 us per 2^20 seeds.)
constexpr uint32_t BUCKET_PT = 8;                 // seeds per thread of the prefix and scatter blocks (256 threads)
constexpr uint32_t BUCKET_BLK = 256 * BUCKET_PT;  // seeds per histogram row
constexpr size_t BUCKET_SMALL_U32 = 260 + 4 + 256;  // offset, n_units, total
inline uint64_t bucket_rows(uint64_t S) { return (S + BUCKET_BLK - 1) / BUCKET_BLK; }
inline size_t bucket_hist_u32(uint64_t S) { return (size_t)(bucket_rows(S) ? bucket_rows(S) : 1) * 256; }
struct Buckets {
    uint32_t *hist;        // [bucket_rows(S)][256]: the blocks' counts, then (k_bucket_colscan) their offsets
    uint32_t *offset;      // [257]
    uint32_t *n_units;     // [1]
    uint32_t *total;       // [256] bucket sizes
    uint4 *units;          // [max_units] {L, start, count, 0}
    uint64_t *sorted_h0;   // [S]
    uint32_t *sorted_idx;  // [S]
};

inline void buckets_small(uint32_t *small, Buckets &b) {
    b.offset = small;
    b.n_units = small + 260;
    b.total = small + 264;
}

// b.hist must already hold the bucket_rows(n_seeds) rows of counts (the caller's prefix kernel, blocks of
// BUCKET_BLK seeds); *zero_word, if given, is zeroed for the caller's work-item counter
int bucket_seeds_counted(hipStream_t st, const uint64_t *d_h0, uint64_t n_seeds, uint32_t seeds_per_unit,
                         Buckets &b, uint32_t *zero_word = nullptr);
// A/B and test knobs: an NMZ_* environment variable is read only when NMZ_AB=1 is set too, so that a production
// process's environment never changes which kernel runs or how a search deals its pairs over ranks
const char *ab_env(const char *name);


}  // namespace nmz
