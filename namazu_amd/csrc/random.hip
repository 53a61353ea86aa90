// K2 -- random-policy fault-injection sweep.
//
// Reference decision (randompolicy.go:300-316,332-346; util/queue/impl.go:94-128):
//   (min,max) = intervals, x0.8 for prioritized entities
//   delay = min == max ? min : rand.Int63n(max-min) + min
//   fault = DefaultFaultAction() != nil && rand.Intn(999) < int(p*1000)
// under the deterministic restatement: each decision
// uses rand.New(rand.NewSource(int64(FNV1a64(le64(seed) || le64(evhash_e)))))
// and draws the delay first, then the fault.
//
// Kernel structure: one seed per lane; seeds bucketed by the low byte of
// their FNV prefix so the per-event FNV correction (same decomposition as
// the replayable sweep, hint = le64(evhash)) is a wave-uniform scalar load;
// the Go seed reduction uses (Hm + Cm - 4*(carry + sign)) mod (2^31-1); the
// first two Go outputs come from closed forms (6 constant modmuls each);
// rejected draws (probability ~1e-7 per Intn(999)) fall back to the general
// closed form y_t, t < 607, per lane.
#include <cstring>

#include "go_rand.h"
#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

constexpr uint64_t MASK63 = 0x7fffffffffffffffULL;
constexpr uint32_t INTN_N = 999;
constexpr uint32_t INT31N_MAX = 0x7fffffffu - (0x80000000u % INTN_N);  // rand.go Int31n

__constant__ uint64_t d_cooked[gorand::LEN] = NMZ_GO_RNG_COOKED_INIT;
[[maybe_unused]] __device__ const gorand::PowTable d_powa = gorand::make_pow_table();
// the same tables for the host decision path (nmz_random_decide_host): the decision code below is shared
[[maybe_unused]] static constexpr gorand::PowTable h_powa = gorand::make_pow_table();
[[maybe_unused]] static constexpr uint64_t h_cooked[gorand::LEN] = NMZ_GO_RNG_COOKED_INIT;
#ifdef __HIP_DEVICE_COMPILE__
#define NMZ_POWA(i) d_powa.v[i]
#define NMZ_COOKED(i) d_cooked[i]
#else
#define NMZ_POWA(i) h_powa.v[i]
#define NMZ_COOKED(i) h_cooked[i]
#endif

// seeded vec[p] for a runtime index (slow path)
__host__ __device__ uint64_t vec_rt(uint32_t s, int p) {
    const uint32_t xa = gorand::modmul(s, NMZ_POWA(21 + 3 * p));
    const uint32_t xb = gorand::modmul(s, NMZ_POWA(22 + 3 * p));
    const uint32_t xc = gorand::modmul(s, NMZ_POWA(23 + 3 * p));
    const uint64_t ck = NMZ_COOKED(p);
    const uint32_t lo = (xb << 20) ^ xc ^ (uint32_t)ck;
    const uint32_t hi = (xa << 8) ^ (xb >> 12) ^ (uint32_t)(ck >> 32);
    return ((uint64_t)hi << 32) | lo;
}

// y_t for 0 <= t < 607: y_t = y_{t-607} + y_{t-273}, y_s (s<0) = vec[(333-s) mod 607]
__host__ __device__ uint64_t go_output(uint32_t s, int t) {
    uint64_t acc = 0;
    int u = t;
    while (u >= 0) {
        acc += vec_rt(s, (333 - (u - 607)) % 607);
        u -= 273;
    }
    return acc + vec_rt(s, ((333 - u) % 607 + 607) % 607);
}

struct ClassParams {
    int64_t min;
    uint64_t n;          // max - min (0 => fixed duration, no draw)
    uint64_t max_accept; // Int63n rejection bound
    uint64_t mu;         // floor(2^64 / n) (Barrett), 0 if n is a power of two
};

struct RandomKParams {
    ClassParams cls[2];
    int32_t fault_threshold;
};

// v mod n for v < 2^63, n not a power of two, mu = floor(2^64/n)
__host__ __device__ __forceinline__ uint64_t mod_barrett(uint64_t v, uint64_t n, uint64_t mu) {
    const uint64_t q = umulhi64(v, mu);
    uint64_t r = v - q * n;
    return r >= n ? r - n : r;
}

struct Decision {
    int64_t delay;
    uint32_t fault;
    uint32_t overflow;
};

// One decision given the reduced Go seed s (1 <= s < 2^31-1) and uniform class bits.
// cp = P.cls[cls & NMZ_EV_PRIORITIZED], selected by the caller (the sweep keeps both classes in SGPRs
// instead of indexing the kernel-argument struct, which costs a scalar load and wait per event)
__host__ __device__ __forceinline__ Decision decide(uint32_t s, uint32_t cls, const ClassParams &cp, int32_t fault_threshold,
                                           uint32_t nm = gorand::NEG_M31) {
    Decision d{0, 0, 0};
    int t = 0;
    if (cp.n) {
        uint64_t v = gorand::out0(s, nm) & MASK63;
        t = 1;
        if (cp.mu) {
            while (v > cp.max_accept) {  // rare: re-draw
                if (t >= gorand::LEN) {
                    d.overflow = 1;
                    break;
                }
                v = go_output(s, t++) & MASK63;
            }
            d.delay = (cp.n >> 31) == 0 ? (int64_t)mod_barrett_small(v, (uint32_t)cp.n, cp.mu) + cp.min
                                        : (int64_t)mod_barrett(v, cp.n, cp.mu) + cp.min;
        } else {
            d.delay = (int64_t)(v & (cp.n - 1)) + cp.min;
        }
    } else {
        d.delay = cp.min;
    }
    if (cls & NMZ_EV_FAULTABLE) {
        if (t == 1) {
            // Intn(999) reads bits 32..62 of y1 = vec[332] + vec[605]: the high words' sum, plus the carry
            // out of the low words. The carry changes v by one, which changes the outcome only when v
            // sits next to the rejection bound or v % 999 next to thr - 1 / 998 (~2e-3 of draws); only
            // then are the low words (two more modmuls) computed.
            const uint32_t v0 = (gorand::vec_hi<332>(s, nm) + gorand::vec_hi<605>(s, nm)) & 0x7fffffffu;
            const uint32_t r0 = v0 % INTN_N;
            if (!(v0 >= INT31N_MAX || r0 == INTN_N - 1 || r0 + 1 == (uint32_t)fault_threshold)) {
                d.fault = ((int32_t)r0 < fault_threshold) ? 1u : 0u;
                return d;
            }
        }
        uint64_t y = (t == 0) ? gorand::out0(s, nm) : (t == 1 ? gorand::out1(s, nm) : go_output(s, t));
        ++t;
        uint32_t v = (uint32_t)(y >> 32) & 0x7fffffffu;
        while (v > INT31N_MAX) {  // rare: re-draw
            if (t >= gorand::LEN) {
                d.overflow = 1;
                break;
            }
            v = (uint32_t)(go_output(s, t++) >> 32) & 0x7fffffffu;
        }
        d.fault = ((int32_t)(v % INTN_N) < fault_threshold) ? 1u : 0u;
    }
    return d;
}

// decide() for the sweep: the same decision with the draw count known per class (0 or 1 Go outputs before the
// fault draw), so that nothing depends on a per-lane draw counter. A lane whose delay or fault draw is rejected
// (probability ~1e-11 and ~3e-7 at the bench parameters) recomputes the whole decision with decide() in a
// divergent branch; a lane whose fault outcome hangs on the low-word carry (~2e-3) computes output 1 in full.
__device__ __forceinline__ Decision decide_sweep(uint32_t s, uint32_t cls, const ClassParams &cp,
                                                 int32_t fault_threshold, uint32_t nm, uint32_t &ovf) {
    Decision d{0, 0, 0};
    bool slow = false;
    if (cp.n) {
        const uint64_t v = gorand::out0(s, nm) & MASK63;
        if (cp.mu) {
            slow = v > cp.max_accept;
            d.delay = (cp.n >> 31) == 0 ? (int64_t)mod_barrett_small(v, (uint32_t)cp.n, cp.mu) + cp.min
                                        : (int64_t)mod_barrett(v, cp.n, cp.mu) + cp.min;
        } else {
            d.delay = (int64_t)(v & (cp.n - 1)) + cp.min;
        }
        if (cls & NMZ_EV_FAULTABLE) {
            const uint32_t v0 = (gorand::vec_hi<332>(s, nm) + gorand::vec_hi<605>(s, nm)) & 0x7fffffffu;
            uint32_t r = v0 % INTN_N;
            if (v0 >= INT31N_MAX || r == INTN_N - 1 || r + 1 == (uint32_t)fault_threshold) {
                const uint32_t v1 = (uint32_t)(gorand::out1(s, nm) >> 32) & 0x7fffffffu;
                slow |= v1 > INT31N_MAX;
                r = v1 % INTN_N;
            }
            d.fault = ((int32_t)r < fault_threshold) ? 1u : 0u;
        }
    } else {
        d.delay = cp.min;
        if (cls & NMZ_EV_FAULTABLE) {
            const uint32_t v = (uint32_t)(gorand::out0(s, nm) >> 32) & 0x7fffffffu;
            slow = v > INT31N_MAX;
            d.fault = ((int32_t)(v % INTN_N) < fault_threshold) ? 1u : 0u;
        }
    }
    if (slow) {  // only here can the Go outputs run out (ovf is updated in this branch alone)
        d = decide(s, cls, cp, fault_threshold, nm);
        ovf |= d.overflow;
    }
    return d;
}

__device__ __forceinline__ uint4 uniform4(uint4 v) {
    return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                      __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}

// Go seed for (prefix state h0 -> H = h0 * P^8, its residue Hm = H mod M31) and
// one table entry q = {C lo, C hi, C mod M31, class}
// nm = -M31 and one = 1 arrive in VGPRs the compiler cannot see through, so that both conditional corrections are
// a VOP2 borrow (v_sub_co) plus a VCC v_cndmask with VGPR operands (full rate) rather than an add of a literal and
// a v_min_u32 (half rate), and the s == 0 test is a borrow out of s - 1 rather than a v_cmp.
__device__ __forceinline__ uint32_t go_seed_from_table(uint64_t H, uint32_t Hm, uint4 q,
                                                       uint32_t nm = gorand::NEG_M31, uint32_t one = 1u) {
    const uint64_t C = ((uint64_t)q.y << 32) | q.x;
    const uint64_t u = H + C;
    const uint32_t k = (uint32_t)(u < H) + (uint32_t)(u >> 63);  // wrap carry + sign
    uint32_t s1 = Hm + q.z, t;                                   // < 2*M31
    s1 = __builtin_sub_overflow(s1, 0u - nm, &t) ? s1 : t;
    uint32_t dd;
    const uint32_t s = __builtin_sub_overflow(s1, 4u * k, &dd) ? dd - nm : dd;
    return __builtin_sub_overflow(s, one, &t) ? 89482311u : s;
}

// per-event table: FNV correction for hint = le64(evhash), class bits
__global__ __launch_bounds__(256) void k_random_table(const uint64_t *__restrict__ evhash,
                                                      const uint8_t *__restrict__ evclass, uint32_t E,
                                                      uint4 *__restrict__ table) {
    const uint32_t e = blockIdx.x, L = threadIdx.x;
    const uint64_t eh = evhash[e];
    uint64_t h = L;
#pragma unroll
    for (int i = 0; i < 8; ++i) h = fnv_step(h, (uint32_t)(eh >> (8 * i)) & 0xff);
    const uint64_t C = h - (uint64_t)L * fnv_pow(8);
    table[(uint64_t)L * E + e] = make_uint4((uint32_t)C, (uint32_t)(C >> 32), (uint32_t)(C % gorand::M31),
                                            evclass[e]);
}

__host__ __device__ __forceinline__ uint64_t seed_prefix(uint64_t seed) {
    uint64_t h = FNV_OFFSET;
#pragma unroll
    for (int i = 0; i < 8; ++i) h = fnv_step(h, (uint32_t)(seed >> (8 * i)) & 0xff);
    return h;
}

__global__ __launch_bounds__(256) void k_random_prefix(uint64_t seed0, uint64_t n, uint64_t *__restrict__ h0,
                                                       uint32_t *__restrict__ rows) {
    // fused bucket histogram (low byte of h0), as in k_seed_prefix: the block's row of `rows` (Buckets)
    constexpr uint32_t ppt = BUCKET_PT;
    __shared__ uint32_t hist[256];
    hist[threadIdx.x] = 0;
    __syncthreads();
    const uint64_t b0 = (uint64_t)blockIdx.x * 256 * ppt;
    for (uint32_t r = 0; r < ppt; ++r) {
        const uint64_t i = b0 + (uint64_t)r * 256 + threadIdx.x;
        if (i < n) {
            const uint64_t h = seed_prefix(seed0 + i);
            h0[i] = h;
            atomicAdd(&hist[h & 0xff], 1u);
        }
    }
    __syncthreads();
    rows[(size_t)blockIdx.x * 256 + threadIdx.x] = hist[threadIdx.x];
}

// Work item = (unit of <= 64 seeds sharing the low byte L, chunk of ec events), handed out by a global atomic
// to a persistent grid. With one wave per unit over all events, 2^20 seeds make 16,640 units for 8,192 wave
// slots: a third round of 256 lone waves took ~5 % of the launch. An item writes its seeds' partial stats
// over [e0, e1) (or the final stats when there is one chunk); k_random_merge combines the chunks in order.
// K32: every delay of both classes lies in [0, 0x7ff00000) ns (host-checked, random_k32), so the running maximum
// is kept as K1 keeps it: the bit pattern of an f64 {lo = ~e, hi = delay}, a non-negative finite double (f64
// denormals are preserved) whose order is (delay, then smaller e) -- the first maximum -- and is updated by one
// v_max_f64 instead of a signed 64-bit compare and three selects; the delay's high word is never formed.
template <bool K32>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_random_sweep(const uint4 *__restrict__ units,
                                                      const uint32_t *__restrict__ n_units,
                                                      const uint64_t *__restrict__ sorted_h0,
                                                      const uint32_t *__restrict__ sorted_idx,
                                                      const uint4 *__restrict__ table, uint32_t E, uint32_t ec,
                                                      uint32_t n_chunks, RandomKParams P,
                                                      uint32_t *__restrict__ item_counter,
                                                      nmz_sched_stats *__restrict__ partial, uint64_t part_stride,
                                                      nmz_sched_stats *__restrict__ stats) {
    const uint32_t lane = threadIdx.x & 63;
    uint32_t nm = gorand::NEG_M31, one = 1u;  // -M and 1 in VGPRs (see gorand::modmul, go_seed_from_table)
    asm volatile("" : "+v"(nm), "+v"(one));
    const uint32_t n_items = *n_units * n_chunks;
    const ClassParams c0 = P.cls[0], c1 = P.cls[1];
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
        const bool active = lane < cnt;
        const uint64_t h0 = active ? sorted_h0[start + lane] : 0;
        const uint64_t H = h0 * fnv_pow(8);
        const uint32_t Hm = (uint32_t)(H % gorand::M31);
        const uint4 *__restrict__ row = table + (uint64_t)L * E;

        uint64_t sum = 0;
        int64_t best = INT64_MIN;
        // argmax = first maximum: starting at the chunk's first event with best = INT64_MIN, a strict >
        // reproduces it (an empty chunk only when E = 0: argmax NMZ_NONE)
        uint32_t arg = e0 < e1 ? e0 : NMZ_NONE, nf = 0, ff = NMZ_NONE, ovf = 0;
        double kmax = 0.0;  // K32: below every real key ({~e, delay} with ~e > 0)
        // the event index is wave-uniform; without the readfirstlane the compiler keeps it in a VGPR
        // (divergent rejection loops below) and loads the entry per lane. The next event's entry is
        // loaded one decision ahead, so its scalar-load latency hides behind the current decision.
        uint4 qn = e0 < e1 ? uniform4(row[__builtin_amdgcn_readfirstlane(e0)]) : make_uint4(0, 0, 0, 0);
        for (uint32_t e = e0; e < e1; ++e) {
            const uint4 q = qn;
            const uint32_t en = __builtin_amdgcn_readfirstlane(min(e + 1, e1 - 1));
            qn = uniform4(row[en]);
            const uint32_t cls = q.w;
            const uint32_t s = go_seed_from_table(H, Hm, q, nm, one);
            const Decision d = decide_sweep(s, cls, (cls & NMZ_EV_PRIORITIZED) ? c1 : c0, P.fault_threshold, nm, ovf);
            if constexpr (K32) {
                const uint32_t d32 = (uint32_t)d.delay;
                sum += d32;
                const double key = __builtin_bit_cast(double, ((uint64_t)d32 << 32) | (uint32_t)~e);
                asm("v_max_f64 %0, %0, %1" : "+v"(kmax) : "v"(key));
            } else {
                sum += (uint64_t)d.delay;
                if (d.delay > best) {
                    best = d.delay;
                    arg = e;
                }
            }
            nf += d.fault;
            ff = min(ff, d.fault ? e : NMZ_NONE);  // events run in increasing order
        }
        if constexpr (K32) {
            if (e0 < e1) {
                const uint64_t kb = __builtin_bit_cast(uint64_t, kmax);
                best = (int64_t)(kb >> 32);
                arg = ~(uint32_t)kb;
            }
        }
        nmz_sched_stats st;
        st.sum_delay_ns = sum;
        st.max_delay_ns = best;
        st.argmax_event = arg;
        st.n_fault = nf;
        st.first_fault = ff;
        st.flags = ovf ? NMZ_STAT_RNG_OVERFLOW : 0u;
        if (n_chunks == 1) {
            if (active) stats[sorted_idx[start + lane]] = st;
        } else {
            partial[(uint64_t)chunk * part_stride + (uint64_t)unit * 64 + lane] = st;
        }
    }
}

// Whether k_random_sweep<true> applies: every delay min + [0, max(n, 1)) of both classes in [0, 0x7ff00000),
// and fewer than 2^32 - 1 events per chunk (~e > 0). NMZ_RANDOM_K32=0 forces the general form.
static bool random_k32(const RandomKParams &kp) {
    static const int env = [] {
        const char *e = ab_env("NMZ_RANDOM_K32");
        return e ? atoi(e) : 1;
    }();
    if (!env) return false;
    for (const ClassParams &c : kp.cls) {
        const uint64_t span = c.n ? c.n : 1;
        if (c.min < 0 || (uint64_t)c.min + span > 0x7ff00000ull) return false;
    }
    return true;
}

// combine the per-chunk partial stats of every seed (in event order) and scatter to the seed's index
__global__ __launch_bounds__(256) void k_random_merge(const uint4 *__restrict__ units,
                                                      const uint32_t *__restrict__ n_units,
                                                      const uint32_t *__restrict__ sorted_idx,
                                                      const nmz_sched_stats *__restrict__ partial,
                                                      uint64_t part_stride, uint32_t n_chunks,
                                                      nmz_sched_stats *__restrict__ stats) {
    const uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    const uint64_t unit = g / 64;
    const uint32_t j = (uint32_t)(g & 63);
    if (unit >= *n_units) return;
    const uint4 u = units[unit];
    if (j >= u.z) return;
    nmz_sched_stats st = partial[g];
    for (uint32_t c = 1; c < n_chunks; ++c) {
        const nmz_sched_stats p = partial[(uint64_t)c * part_stride + g];
        st.sum_delay_ns += p.sum_delay_ns;
        if (p.max_delay_ns > st.max_delay_ns) {
            st.max_delay_ns = p.max_delay_ns;
            st.argmax_event = p.argmax_event;
        }
        st.n_fault += p.n_fault;
        if (st.first_fault == NMZ_NONE) st.first_fault = p.first_fault;
        st.flags |= p.flags;
    }
    stats[sorted_idx[u.y + j]] = st;
}

__global__ __launch_bounds__(256) void k_random_dump(uint64_t seed0, uint64_t n_dump, const uint4 *__restrict__ table,
                                                     uint32_t E, RandomKParams P, int64_t *__restrict__ delays,
                                                     uint8_t *__restrict__ faults, uint32_t *__restrict__ overflow) {
    uint64_t idx = (uint64_t)blockIdx.x * 256 + threadIdx.x;
    if (idx >= n_dump * E) return;
    const uint64_t sidx = idx / E;
    const uint32_t e = (uint32_t)(idx % E);
    const uint64_t h0 = seed_prefix(seed0 + sidx);
    const uint64_t H = h0 * fnv_pow(8);
    const uint4 q = table[(h0 & 0xff) * E + e];
    // direct form: int64 seed, Go's reduction, no residue shortcut
    const uint64_t u = H + (((uint64_t)q.y << 32) | q.x);
    const uint32_t s = gorand::seed_reduce((int64_t)u);
    const Decision d = decide(s, q.w, P.cls[q.w & NMZ_EV_PRIORITIZED], P.fault_threshold);
    delays[idx] = d.delay;
    faults[idx] = (uint8_t)d.fault;
    if (d.overflow) atomicOr(overflow, 1u);
}

// online decisions for one seed (QueueEvent): one thread per pending event, the direct form of k_random_dump
// without a table -- FNV over le64(seed) || le64(evhash), Go's seed reduction, decide()
__global__ __launch_bounds__(256) void k_random_decide(uint64_t seed, const uint64_t *__restrict__ evhash,
                                                       const uint8_t *__restrict__ evclass, uint32_t n,
                                                       RandomKParams P, int64_t *__restrict__ delays,
                                                       uint8_t *__restrict__ faults, uint32_t *__restrict__ overflow) {
    const uint32_t e = blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    uint64_t h = seed_prefix(seed);
    const uint64_t eh = evhash[e];
#pragma unroll
    for (int i = 0; i < 8; ++i) h = fnv_step(h, (uint32_t)(eh >> (8 * i)) & 0xff);
    const uint32_t s = gorand::seed_reduce((int64_t)h);
    const uint32_t cls = evclass[e];
    const Decision d = decide(s, cls, P.cls[cls & NMZ_EV_PRIORITIZED], P.fault_threshold);
    delays[e] = d.delay;
    faults[e] = (uint8_t)d.fault;
    if (d.overflow) atomicOr(overflow, 1u);
}

}  // namespace nmz

struct nmz_random_plan {
    nmz_ctx *ctx = nullptr;
    uint32_t n_events = 0;
    nmz::RandomKParams kp{};
    uint4 *d_table = nullptr;
    uint64_t max_seeds = 0;
    nmz::DevBuf table_mem;
    nmz::DevBuf seed_scratch;
    nmz::DevBuf partial;  // per-chunk partial stats per seed slot (n_chunks > 1)
};

namespace nmz {

static int make_kparams(const nmz_random_params *p, RandomKParams &kp) {
    NMZ_CHECK(p != nullptr, "params is NULL");
    std::memset(&kp, 0, sizeof kp);
    for (int i = 0; i < 2; ++i) {
        NMZ_CHECK(p->min_ns[i] <= p->max_ns[i], "minDuration > maxDuration (util/queue/impl.go:36)");
        ClassParams &c = kp.cls[i];
        c.min = p->min_ns[i];
        c.n = (uint64_t)(p->max_ns[i] - p->min_ns[i]);
        if (c.n) {
            NMZ_CHECK(c.n <= (uint64_t)INT64_MAX, "interval span exceeds int64");
            if ((c.n & (c.n - 1)) == 0) {
                c.mu = 0;
                c.max_accept = UINT64_MAX;
            } else {
                c.mu = (uint64_t)(((unsigned __int128)1 << 64) / c.n);
                c.max_accept = (uint64_t)INT64_MAX - ((1ULL << 63) % c.n);  // rand.go Int63n
            }
        }
    }
    kp.fault_threshold = p->fault_threshold;
    return NMZ_OK;
}

// Events per work item. 2^20 seeds x 10^4 events: 512 -> 26.0 ms, 1,024 -> 26.2, 2,048 -> 26.5 (the last round of
// work items is shorter with small items). 10^7 seeds: 512 / 1,024 / 2,048 all 245-246 ms, but each chunk adds a
// 32-byte partial row per seed (written by the sweep, read by k_random_merge): 2,048 keeps that to 5 rows per seed
// (8.1 -> ~2 GB per launch). NMZ_RANDOM_EC overrides.
constexpr uint32_t RANDOM_EC = 512;
constexpr uint32_t RANDOM_EC_LARGE = 2048;        // from RANDOM_EC_LARGE_SEEDS seeds per launch
constexpr uint64_t RANDOM_EC_LARGE_SEEDS = 1ULL << 22;

static uint32_t random_ec(uint64_t S) {
    static const uint32_t env = [] {
        const char *e = ab_env("NMZ_RANDOM_EC");
        const uint32_t x = e ? (uint32_t)atoi(e) : 0u;
        return x >= 64 ? x : 0u;
    }();
    return env ? env : (S >= RANDOM_EC_LARGE_SEEDS ? RANDOM_EC_LARGE : RANDOM_EC);
}

static size_t random_seed_scratch_bytes(uint64_t S) {
    return Carve::bytes_for(S, 8) * 2 + Carve::bytes_for(S, 4) + Carve::bytes_for(BUCKET_SMALL_U32, 4) +
           Carve::bytes_for(bucket_hist_u32(S), 4) + Carve::bytes_for(S / 64 + 257, 16) + Carve::bytes_for(4, 4);
}

static Buckets carve_random(void *p, uint64_t S, uint64_t **h0, uint32_t **counter) {
    Carve cv(p);
    *h0 = cv.take<uint64_t>(S);
    Buckets b;
    b.sorted_h0 = cv.take<uint64_t>(S);
    b.sorted_idx = cv.take<uint32_t>(S);
    buckets_small(cv.take<uint32_t>(BUCKET_SMALL_U32), b);
    b.hist = cv.take<uint32_t>(bucket_hist_u32(S));
    b.units = cv.take<uint4>(S / 64 + 257);
    *counter = cv.take<uint32_t>(4);
    return b;
}

static int random_plan_create(nmz_ctx *ctx, const uint64_t *evhash, const uint8_t *evclass, uint32_t E,
                              const nmz_random_params *params, uint64_t max_seeds, nmz_random_plan **out) {
    NMZ_CHECK(ctx && out, "NULL argument");
    NMZ_CHECK(E == 0 || (evhash && evclass), "evhash/evclass is NULL");
    for (uint32_t e = 0; e < E; ++e)
        NMZ_CHECK((evclass[e] & ~(NMZ_EV_PRIORITIZED | NMZ_EV_FAULTABLE)) == 0,
                  "evclass has unknown bits (ProcSetEvent decisions are out of scope)");
    RandomKParams kp;
    NMZ_TRY(make_kparams(params, kp));
    auto *p = new nmz_random_plan();
    p->ctx = ctx;
    p->n_events = E;
    p->kp = kp;
    p->max_seeds = max_seeds;
    hipStream_t st = ctx->stream;
    auto cleanup = [&](int code) {
        p->table_mem.release();
        p->seed_scratch.release();
        p->partial.release();
        delete p;
        return code;
    };
    int rc = p->table_mem.ensure(Carve::bytes_for((size_t)256 * E + 1, 16) + Carve::bytes_for(E + 1, 8) +
                                 Carve::bytes_for(E + 1, 1));
    if (rc == NMZ_OK) rc = p->seed_scratch.ensure(random_seed_scratch_bytes(max_seeds));
    if (rc != NMZ_OK) return cleanup(rc);
    Carve cv(p->table_mem.ptr);
    p->d_table = cv.take<uint4>((size_t)256 * E + 1);
    uint64_t *d_eh = cv.take<uint64_t>(E + 1);
    uint8_t *d_ec = cv.take<uint8_t>(E + 1);
    if (E) {
        if (hipMemcpyAsync(d_eh, evhash, (size_t)E * 8, hipMemcpyHostToDevice, st) ||
            hipMemcpyAsync(d_ec, evclass, E, hipMemcpyHostToDevice, st))
            return cleanup(fail(NMZ_EHIP, "plan upload failed"));
        hipLaunchKernelGGL(k_random_table, dim3(E), dim3(256), 0, st, d_eh, d_ec, E, p->d_table);
        if (hipGetLastError() != hipSuccess || hipStreamSynchronize(st) != hipSuccess)
            return cleanup(fail(NMZ_EHIP, "random table kernel failed"));
    }
    *out = p;
    return NMZ_OK;
}

static int random_run(nmz_random_plan *p, hipStream_t st, uint64_t seed0, uint64_t S, nmz_sched_stats *d_stats) {
    if (S == 0) return NMZ_OK;
    NMZ_CHECK(S <= p->max_seeds, "more seeds than the plan was created for");
    const uint32_t E = p->n_events;
    uint64_t *d_h0;
    uint32_t *d_counter;
    Buckets b = carve_random(p->seed_scratch.ptr, p->max_seeds, &d_h0, &d_counter);
    hipLaunchKernelGGL(k_random_prefix, dim3(ceil_div(S, BUCKET_BLK)), dim3(256), 0, st, seed0, S, d_h0, b.hist);
    const uint64_t max_units = S / 64 + 256;
    NMZ_TRY(bucket_seeds_counted(st, d_h0, S, 64, b, d_counter));
    const uint32_t ec = random_ec(S);
    const uint32_t n_chunks = std::max<uint32_t>(1, (E + ec - 1) / ec);
    const uint64_t stride = (p->max_seeds / 64 + 257) * 64;
    nmz_sched_stats *part = nullptr;
    if (n_chunks > 1) {
        NMZ_TRY(p->partial.ensure(Carve::bytes_for(stride * n_chunks, sizeof(nmz_sched_stats))));
        part = p->partial.as<nmz_sched_stats>();
    }
    const unsigned grid = (unsigned)std::min<uint64_t>(p->ctx->n_cu * 8ull, ceil_div(max_units * n_chunks, 4));
    {
        KernelTimer kt(p->ctx, st, "random_sweep");
        if (random_k32(p->kp))
            hipLaunchKernelGGL(k_random_sweep<true>, dim3(grid), dim3(256), 0, st, b.units, b.n_units, b.sorted_h0,
                               b.sorted_idx, p->d_table, E, ec, n_chunks, p->kp, d_counter, part, stride, d_stats);
        else
            hipLaunchKernelGGL(k_random_sweep<false>, dim3(grid), dim3(256), 0, st, b.units, b.n_units,
                               b.sorted_h0, b.sorted_idx, p->d_table, E, ec, n_chunks, p->kp, d_counter, part,
                               stride, d_stats);
    }
    if (n_chunks > 1)
        hipLaunchKernelGGL(k_random_merge, dim3(ceil_div(max_units * 64, 256)), dim3(256), 0, st, b.units,
                           b.n_units, b.sorted_idx, part, stride, n_chunks, d_stats);
    NMZ_HIP(hipGetLastError());
    return NMZ_OK;
}

}  // namespace nmz

using namespace nmz;

extern "C" {

int nmz_random_plan_create(nmz_ctx *ctx, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                           const nmz_random_params *params, uint64_t max_seeds, nmz_random_plan **out) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    NMZ_CHECK(max_seeds < (1ULL << 32), "at most 2^32-1 seeds per plan");
    return random_plan_create(ctx, evhash, evclass, n_events, params, max_seeds, out);
}

int nmz_random_plan_destroy(nmz_random_plan *plan) {
    if (!plan) return NMZ_OK;
    {
        CtxGuard g(plan->ctx);
        plan->table_mem.release();
        plan->seed_scratch.release();
        plan->partial.release();
    }
    delete plan;
    return NMZ_OK;
}

int nmz_random_sweep_dev(nmz_random_plan *plan, uint64_t seed0, uint64_t n_seeds, nmz_sched_stats *d_stats,
                         void *stream) {
    NMZ_CHECK(plan != nullptr, "plan is NULL");
    CtxGuard g(plan->ctx);
    NMZ_TRY(g.rc);
    return random_run(plan, stream ? (hipStream_t)stream : plan->ctx->stream, seed0, n_seeds, d_stats);
}

int nmz_random_sweep(nmz_ctx *ctx, uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash, const uint8_t *evclass,
                     uint32_t n_events, const nmz_random_params *params, nmz_sched_stats *stats, int64_t *delays,
                     uint8_t *faults, uint64_t n_dump_seeds, uint32_t k, nmz_topk_entry *topk) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    NMZ_CHECK(n_dump_seeds <= n_seeds, "n_dump_seeds > n_seeds");
    NMZ_CHECK(n_seeds < (1ULL << 32), "at most 2^32-1 seeds per call");
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    hipStream_t st = ctx->stream;
    nmz_random_plan *plan = nullptr;
    NMZ_TRY(random_plan_create(ctx, evhash, evclass, n_events, params, n_seeds, &plan));
    struct PlanGuard {
        nmz_random_plan *p;
        ~PlanGuard() {
            p->table_mem.release();
            p->seed_scratch.release();
            p->partial.release();
            delete p;
        }
    } pg{plan};
    const uint64_t nd = n_dump_seeds * n_events;
    const uint64_t tk_entries = topk_scratch_entries(n_seeds, k);
    size_t need = Carve::bytes_for(n_seeds + 1, sizeof(nmz_sched_stats)) + Carve::bytes_for(nd + 1, 8) +
                  Carve::bytes_for(nd + 1, 1) + Carve::bytes_for(4, 4) + Carve::bytes_for(tk_entries + k + 1, 24);
    NMZ_TRY(ctx->buf[1].ensure(need));
    Carve cv(ctx->buf[1].ptr);
    nmz_sched_stats *d_stats = cv.take<nmz_sched_stats>(n_seeds + 1);
    int64_t *d_del = cv.take<int64_t>(nd + 1);
    uint8_t *d_flt = cv.take<uint8_t>(nd + 1);
    uint32_t *d_ovf = cv.take<uint32_t>(4);
    nmz_topk_entry *d_tk = cv.take<nmz_topk_entry>(tk_entries + k + 1);
    NMZ_HIP(hipMemsetAsync(d_ovf, 0, 4, st));
    if (n_events == 0) {
        for (uint64_t i = 0; i < n_seeds && stats; ++i) stats_empty(stats[i]);
    }
    if (n_events) NMZ_TRY(random_run(plan, st, seed0, n_seeds, d_stats));
    if (nd) {
        hipLaunchKernelGGL(k_random_dump, dim3(ceil_div(nd, 256)), dim3(256), 0, st, seed0, n_dump_seeds,
                           plan->d_table, n_events, plan->kp, d_del, d_flt, d_ovf);
        NMZ_HIP(hipGetLastError());
    }
    if (k && n_events) NMZ_TRY(topk_select(st, d_stats, n_seeds, seed0, k, d_tk, d_tk + tk_entries));
    uint32_t ovf = 0;
    if (stats && n_seeds && n_events)
        NMZ_HIP(hipMemcpyAsync(stats, d_stats, n_seeds * sizeof(nmz_sched_stats), hipMemcpyDeviceToHost, st));
    if (delays && nd) NMZ_HIP(hipMemcpyAsync(delays, d_del, nd * 8, hipMemcpyDeviceToHost, st));
    if (faults && nd) NMZ_HIP(hipMemcpyAsync(faults, d_flt, nd, hipMemcpyDeviceToHost, st));
    if (topk && k && n_events)
        NMZ_HIP(hipMemcpyAsync(topk, d_tk + tk_entries, k * sizeof(nmz_topk_entry), hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    if (ovf) return fail(NMZ_ERANGE, "a decision needed more than 607 Go rng outputs");
    if (topk && k && n_events == 0) {
        // no events: every seed ties at (0 faults, sum 0) -> smallest seeds first
        for (uint32_t i = 0; i < k; ++i) {
            if (i < n_seeds) {
                topk[i].seed = seed0 + i;
                topk[i].sum_delay_ns = 0;
                topk[i].n_fault = 0;
                topk[i].first_fault = NMZ_NONE;
            } else {
                topk[i].seed = UINT64_MAX;
                topk[i].sum_delay_ns = INT64_MIN;
                topk[i].n_fault = 0;
                topk[i].first_fault = NMZ_NONE;
            }
        }
    }
    return NMZ_OK;
}

// Online decisions on the calling host thread (Random.QueueEvent decides at enqueue, util/queue/impl.go:35-46,
// 110-128): the same FNV, seed reduction and decide() closed forms the kernels run (shared __host__ __device__
// code above), one event at a time, no device work.
int nmz_random_decide_host(uint64_t seed, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                           const nmz_random_params *params, int64_t *delays, uint8_t *faults) {
    RandomKParams kp;
    NMZ_TRY(make_kparams(params, kp));
    if (n_events == 0) return NMZ_OK;
    NMZ_CHECK(evhash && evclass && delays && faults, "NULL argument");
    const uint64_t h0 = seed_prefix(seed);
    for (uint32_t e = 0; e < n_events; ++e) {
        const uint32_t cls = evclass[e];
        NMZ_CHECK((cls & ~(NMZ_EV_PRIORITIZED | NMZ_EV_FAULTABLE)) == 0,
                  "evclass has unknown bits (ProcSetEvent decisions are out of scope)");
        uint64_t h = h0;
        for (int i = 0; i < 8; ++i) h = fnv_step(h, (uint32_t)(evhash[e] >> (8 * i)) & 0xff);
        const Decision d = decide(gorand::seed_reduce((int64_t)h), cls, kp.cls[cls & NMZ_EV_PRIORITIZED],
                                  kp.fault_threshold);
        if (d.overflow) return fail(NMZ_ERANGE, "a decision needed more than 607 Go rng outputs");
        delays[e] = d.delay;
        faults[e] = (uint8_t)d.fault;
    }
    return NMZ_OK;
}

// Online decisions for one seed (Random.QueueEvent -> makeActionForEvent, randompolicy.go:300-346 +
// util/queue/impl.go:94-128, under the DESIGN.md section 2 contract): a batch of n pending events, no plan.
int nmz_random_decide(nmz_ctx *ctx, uint64_t seed, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                      const nmz_random_params *params, int64_t *delays, uint8_t *faults) {
    NMZ_CHECK(ctx != nullptr, "ctx is NULL");
    RandomKParams kp;
    NMZ_TRY(make_kparams(params, kp));
    CtxGuard g(ctx);
    NMZ_TRY(g.rc);
    if (n_events == 0) return NMZ_OK;
    NMZ_CHECK(evhash && evclass && delays && faults, "NULL argument");
    for (uint32_t e = 0; e < n_events; ++e)
        NMZ_CHECK((evclass[e] & ~(NMZ_EV_PRIORITIZED | NMZ_EV_FAULTABLE)) == 0,
                  "evclass has unknown bits (ProcSetEvent decisions are out of scope)");
    hipStream_t st = ctx->stream;
    NMZ_TRY(ctx->buf[9].ensure(Carve::bytes_for(n_events, 8) * 2 + Carve::bytes_for(n_events, 1) * 2 +
                               Carve::bytes_for(4, 4)));
    Carve cv(ctx->buf[9].ptr);
    uint64_t *d_eh = cv.take<uint64_t>(n_events);
    int64_t *d_del = cv.take<int64_t>(n_events);
    uint8_t *d_ec = cv.take<uint8_t>(n_events);
    uint8_t *d_flt = cv.take<uint8_t>(n_events);
    uint32_t *d_ovf = cv.take<uint32_t>(4);
    NMZ_HIP(hipMemsetAsync(d_ovf, 0, 4, st));
    NMZ_HIP(hipMemcpyAsync(d_eh, evhash, (uint64_t)n_events * 8, hipMemcpyHostToDevice, st));
    NMZ_HIP(hipMemcpyAsync(d_ec, evclass, n_events, hipMemcpyHostToDevice, st));
    hipLaunchKernelGGL(k_random_decide, dim3(ceil_div(n_events, 256)), dim3(256), 0, st, seed, d_eh, d_ec, n_events,
                       kp, d_del, d_flt, d_ovf);
    NMZ_HIP(hipGetLastError());
    uint32_t ovf = 0;
    NMZ_HIP(hipMemcpyAsync(delays, d_del, (uint64_t)n_events * 8, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipMemcpyAsync(faults, d_flt, n_events, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipMemcpyAsync(&ovf, d_ovf, 4, hipMemcpyDeviceToHost, st));
    NMZ_HIP(hipStreamSynchronize(st));
    if (ovf) return fail(NMZ_ERANGE, "a decision needed more than 607 Go rng outputs");
    return NMZ_OK;
}

}  // extern "C"
