/*
 * nmz_gpu.h -- C ABI of libnmz_gpu.so, the MI355X (gfx950) engine behind
 * Namazu's explore-policy decision path and historystorage similarity search.
 *
 * This is the drop-in boundary: plain pointers and sizes, no HIP or torch
 * types, every call returns an int status (NMZ_OK == 0, <0 on error, message
 * in nmz_last_error()). A Go host binds it through cgo;
 * the Python host mirror in namazu_amd/ binds it through ctypes.
 *
 * Reference interfaces each entry point replaces (paths relative to the
 * reference tree, nmz/):
 *
 *   nmz_replayable_sweep*  -> Replayable.determineInterval / QueueEvent
 *                             explorepolicy/replayable/replayablepolicy.go:100-126
 *                             (FNV-1a64(seed || hint) % maxInterval), batched over
 *                             seeds x events.
 *   nmz_random_sweep*      -> Random.QueueEvent + makeActionForEvent
 *                             explorepolicy/random/randompolicy.go:300-316,332-346
 *                             + util/queue/impl.go:35-46,94-128 (Int63n delay,
 *                             Intn(999) fault draw), batched over seeds x events
 *                             under the deterministic per-event seeding contract
 *                             documented in DESIGN.md section 2.
 *   nmz_random_params_resolve -> Random.LoadConfig's interval/probability
 *                             semantics randompolicy.go:156-228,332-340.
 *   nmz_ed_pairs / nmz_ed_allpairs_knn -> HistoryStorage similarity search
 *                             (optional interface next to Search /
 *                             SearchWithConverter, historystorage/historystorage.go:50-51,
 *                             naive/naive.go:235-257); distance 0 <=> SingleTrace.Equals
 *                             (util/trace/trace.go:29-31).
 *
 * Buffers passed to the host-pointer entry points are borrowed for the call
 * only and never retained (cgo pointer rules). The *_dev entry points take
 * device pointers that are already resident in HBM plus a hipStream_t passed
 * as void*; they enqueue asynchronously on that stream.
 *
 * Threading: a context is bound to one device; calls on one context are
 * serialized by a mutex inside it and call hipSetDevice on entry, so a Go
 * caller may invoke them from any OS thread.
 */
#ifndef NMZ_GPU_H
#define NMZ_GPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NMZ_ABI_VERSION 1

/* status codes */
#define NMZ_OK 0
#define NMZ_EINVAL (-1)   /* bad argument (mirrors LoadConfig errors / queue panics) */
#define NMZ_EHIP (-2)     /* HIP runtime error */
#define NMZ_ENOMEM (-3)   /* device allocation failed */
#define NMZ_ERANGE (-4)   /* a decision needed more Go rng outputs than the kernel's closed form covers */
#define NMZ_EAGAIN (-5)   /* nothing became ready within the timeout (nmz_tbqueue_dequeue) */

/* per-event class bits for the random policy (one uint8 per event) */
#define NMZ_EV_PRIORITIZED 0x01u /* EntityID() in prioritizedEntities (randompolicy.go:335) */
#define NMZ_EV_FAULTABLE 0x02u   /* DefaultFaultAction() != nil: deferred Packet/Filesystem
                                    event (event_packet.go:45-47, event_filesystem.go:58-60) */

/* stats flags */
#define NMZ_STAT_RNG_OVERFLOW 0x01u

#define NMZ_NONE 0xffffffffu

/* Per-schedule statistics (one per seed), 32 bytes.
 * delays are time.Duration values (int64 ns). */
typedef struct nmz_sched_stats {
    uint64_t sum_delay_ns;  /* sum of delays, mod 2^64 (two's complement)          */
    int64_t max_delay_ns;   /* max delay (signed); INT64_MIN when there are no events */
    uint32_t argmax_event;  /* first event attaining max_delay_ns; NMZ_NONE if none */
    uint32_t n_fault;       /* number of fault actions chosen                        */
    uint32_t first_fault;   /* first event given a fault action; NMZ_NONE if none    */
    uint32_t flags;         /* NMZ_STAT_* bits                                       */
} nmz_sched_stats;

/* Failure-schedule candidate, ordered by (n_fault desc, sum_delay desc as int64,
 * seed asc). */
typedef struct nmz_topk_entry {
    uint64_t seed;
    int64_t sum_delay_ns;
    uint32_t n_fault;
    uint32_t first_fault;
} nmz_topk_entry;

/* Resolved random-policy parameters: the kernel consumes integers only.
 * Index 0 = ordinary entity, 1 = prioritized entity (x0.8 intervals). */
typedef struct nmz_random_params {
    int64_t min_ns[2];
    int64_t max_ns[2];
    int32_t fault_threshold; /* int(faultActionProbability * 1000.0) */
    uint32_t reserved;
} nmz_random_params;

typedef struct nmz_ctx nmz_ctx;

/* ---- context ---------------------------------------------------------- */
int nmz_open(int device, nmz_ctx **out);
int nmz_close(nmz_ctx *ctx);
const char *nmz_last_error(void); /* thread-local, valid until the next call on this thread */
int nmz_abi_version(void);
int nmz_device_count(int *count);
/* The context's own stream (hipStream_t as void*): what a NULL stream argument of the *_dev entry points means.
 * Each context's stream is created by the library (hipStreamCreateWithFlags), so contexts' streams are distinct
 * streams a caller may pipeline over (one plan per stream) and order its own work against. */
int nmz_ctx_stream(nmz_ctx *ctx, void **stream);

/* Kernel timing (HIP events recorded on the launch stream around the dominant
 * kernels: "replayable_sweep", "random_sweep", "ed_tile"). on = 0 off, 1 events and
 * spans, NMZ_TIMING_SPANS (2) the kernels' own spans only (no event records between a
 * stream's launches: each record is a marker the queue waits on, ~6 us). */
#define NMZ_TIMING_SPANS 2
int nmz_timing_enable(nmz_ctx *ctx, int on);
int nmz_timing_read(nmz_ctx *ctx, const char *kernel, double *total_ms, uint64_t *count, int reset);
/* The same kernels' execution spans as the kernels record them (first workgroup start to last workgroup end,
 * wall_clock64()), so launches that wait on the stream for another stream's kernels are not charged the
 * wait ("replayable_sweep" on the order-query path): total_ms = the length of the union of the spans
 * (launches that overlap share their common time), count = launches. reset clears every kernel's spans. */
int nmz_timing_read_span(nmz_ctx *ctx, const char *kernel, double *total_ms, uint64_t *count, int reset);

/* FNV-1a 64 of each of n byte strings (CSR off[n+1] into bytes), one thread per string: the event
 * identities of a batch of events (their canonical JSON; Go hash/fnv New64a). */
int nmz_fnv1a64_batch(nmz_ctx *ctx, const uint64_t *off, const uint8_t *bytes, uint64_t n, uint64_t *out);

/* ---- online decisions on the calling host thread (no device work) ------------------------------------
 * The reference decides at enqueue, in the caller's goroutine (util/queue/impl.go:35-46,110-128;
 * replayablepolicy.go:116-126), and QueueEvent must not block (randompolicy_test.go:112-118): a GPU launch per
 * event (~100 us) is longer than the decision itself, so the online path decides on the host with the same
 * closed forms the kernels run (shared code: FNV, Go's seed reduction, the jump-ahead rngSource outputs,
 * Int63n / Intn rejection). Results equal nmz_*_decide and the sweeps bit for bit. Batch work (sweeps,
 * all-pairs search) stays on the GPU. */
int nmz_random_decide_host(uint64_t seed, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                           const nmz_random_params *params, int64_t *delays, uint8_t *faults);
int nmz_replayable_decide_host(const uint8_t *seed, uint32_t seed_len, const uint32_t *hint_off,
                               const uint8_t *hint_bytes, uint32_t n_events, int64_t max_interval_ns,
                               int64_t *delays);
/* FNV-1a 64 of n byte strings (an event's canonical JSON -> its identity) */
int nmz_fnv1a64_batch_host(const uint64_t *off, const uint8_t *bytes, uint64_t n, uint64_t *out);

/* Time-bounded queue (util/queue/impl.go:64-128 BasicTBQueue; host only). One timer thread releases two kinds of
 * item, times in CLOCK_MONOTONIC ns (nmz_monotonic_ns):
 *   nmz_tbqueue_enqueue       a ranged item (min != max, impl.go:120-126): released at due_ns = enqueue + its drawn
 *                             duration;
 *   nmz_tbqueue_enqueue_fixed a fixed-duration item (min == max, impl.go:77-89,117-119): one FIFO lane whose head is
 *                             released at max(its enqueue, the previous fixed item's release) + duration, so a burst
 *                             of n items of duration d leaves at d, 2d, ..., nd, in enqueue order.
 * Equal due times release in enqueue order; consumers block in dequeue (the policy's ActionChan). A released item
 * records its due and release times, so release - due is the delivered-delay error of the online path. */
typedef struct nmz_tbqueue nmz_tbqueue;
int nmz_tbqueue_create(nmz_tbqueue **out);
/* close: no further enqueues; every consumer blocked in dequeue (and every later dequeue) returns NMZ_EAGAIN.
 * destroy: closes, joins the timer thread, waits until no call is inside dequeue, then frees the queue. A caller
 * must not start a call on the queue once destroy has begun (close first, let the consumers return, then
 * destroy: namazu_amd/explorepolicy.py ActionChannel.close). */
int nmz_tbqueue_close(nmz_tbqueue *q);
int nmz_tbqueue_destroy(nmz_tbqueue *q);
int64_t nmz_monotonic_ns(void);
int nmz_tbqueue_enqueue(nmz_tbqueue *q, uint64_t id, int64_t due_ns);
int nmz_tbqueue_enqueue_fixed(nmz_tbqueue *q, uint64_t id, int64_t enqueued_ns, int64_t duration_ns);
/* timeout_ns < 0: wait forever; NMZ_EAGAIN when nothing was released in time */
int nmz_tbqueue_dequeue(nmz_tbqueue *q, int64_t timeout_ns, uint64_t *id, int64_t *due_ns, int64_t *released_ns);
int nmz_tbqueue_stats(nmz_tbqueue *q, uint64_t *enqueued, uint64_t *released, uint64_t *dequeued);

/* ---- parameter resolution (host only, no device work) -------------------
 * min/max are time.Duration ns as parsed by LoadConfig; probability as float64.
 * Applies the prioritized x0.8 truncation in IEEE double exactly like
 * randompolicy.go:337-339, the threshold int(p*1000.0) of :310, and the
 * validity checks of :223-225 (probability) and util/queue/impl.go:36-38
 * (min > max). */
int nmz_random_params_resolve(int64_t min_ns, int64_t max_ns, double fault_probability,
                              nmz_random_params *out);

/* ---- replayable policy sweep ------------------------------------------
 * For each seed s (CSR: seed_off[n_seeds+1] into seed_bytes) and event e
 * (CSR: hint_off[n_events+1] into hint_bytes, the events' ReplayHint()):
 *     delay[s][e] = int64( FNV1a64(seed_s || hint_e) % uint64(max_interval_ns) )
 * and 0 for every event when max_interval_ns == 0 (replayablepolicy.go:101-104).
 * Outputs (each may be NULL):
 *   stats[n_seeds]
 *   delays[n_dump_seeds * n_events]  row-major, for the first n_dump_seeds seeds
 *   topk[k]   best k seeds by (sum_delay desc, seed index asc); entry .seed is
 *             the seed's index in the CSR.                                    */
int nmz_replayable_sweep(nmz_ctx *ctx, const uint32_t *seed_off, const uint8_t *seed_bytes,
                         uint64_t n_seeds, const uint32_t *hint_off, const uint8_t *hint_bytes,
                         uint32_t n_events, int64_t max_interval_ns, nmz_sched_stats *stats,
                         int64_t *delays, uint64_t n_dump_seeds, uint32_t k,
                         nmz_topk_entry *topk);

/* Device-resident variant (all pointers are device pointers; hipStream_t as void*).
 * The plan holds the per-event tables of one hint table and the scratch of one sweep
 * for up to max_seeds seeds. Sweeps through one plan must be ordered (one stream at a
 * time); concurrent sweeps on several streams take one plan each (bench.py pipelines
 * three). */
typedef struct nmz_replayable_plan nmz_replayable_plan;
int nmz_replayable_plan_create(nmz_ctx *ctx, const uint32_t *hint_off, const uint8_t *hint_bytes,
                               uint32_t n_events, int64_t max_interval_ns,
                               uint64_t max_seeds, nmz_replayable_plan **out);
/* The same, returning as soon as the build is enqueued on the context's stream (the host arrays may be
 * reused at once: they are staged in pinned memory). A sweep through the plan on any stream waits for the
 * build on the device; destroy waits for it and for the plan's sweeps. For a stream of traces: create trace
 * i + 1's plan (on a second context, so its build overlaps) while trace i sweeps. Plans the wavelet-tree plan
 * kernel does not build in one launch (a class of 4,096 events or more, order-query or per-decision plans)
 * are built synchronously as by nmz_replayable_plan_create. */
int nmz_replayable_plan_create_async(nmz_ctx *ctx, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                     uint32_t n_events, int64_t max_interval_ns, uint64_t max_seeds,
                                     nmz_replayable_plan **out);
/* A prepared seed set for sweeping one set of seeds over many traces' plans: the seeds' prefix hashes (FNV of the
 * seed bytes), bucketed by table row once, instead of per sweep. d_seed_off / d_seed_bytes: device CSR of the seed
 * strings, or d_seed_off == NULL: the decimal strings of dec_lo .. dec_lo + n_seeds - 1. Synchronous; the set may be
 * swept through any plan on the same device and stream (results identical to nmz_replayable_sweep_topk_dev and
 * nmz_replayable_sweep_decimal_topk_dev over the same seeds). Destroy waits for the device. */
typedef struct nmz_replayable_seeds nmz_replayable_seeds;
int nmz_replayable_seeds_create(nmz_ctx *ctx, const uint32_t *d_seed_off, const uint8_t *d_seed_bytes,
                                uint64_t n_seeds, uint64_t dec_lo, nmz_replayable_seeds **out);
int nmz_replayable_seeds_destroy(nmz_replayable_seeds *seeds);
/* nmz_replayable_sweep_topk_dev over a prepared seed set: stats for every seed of the set, and (k > 0) the top-k
 * with seed = seed0 + the seed's index. */
int nmz_replayable_sweep_seeds_topk_dev(nmz_replayable_plan *plan, const nmz_replayable_seeds *seeds, uint64_t seed0,
                                        uint32_t k, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk, void *stream);
/* A batch of recorded traces over one decimal seed range (the reference seeds "lo" .. "lo + n - 1",
 * replayablepolicy.go:74-87): for every trace t (hint CSR hint_off[t] / hint_bytes[t], n_events[t] hints) its own
 * plan, the sweep of all n_seeds seeds and the top-k failure candidates into topk[t * k .. t * k + k) (as
 * nmz_replayable_sweep_decimal_topk_dev). Pipelined inside: the seeds are prepared once, trace t + 2's plan builds
 * while trace t sweeps (on a private second context the call opens on first use), top-k lists come back while
 * the next trace sweeps. Host arrays only; synchronous. 1 <= k <= 256. */
int nmz_replayable_sweep_traces(nmz_ctx *ctx, uint32_t n_traces, const uint32_t *const *hint_off,
                                const uint8_t *const *hint_bytes, const uint32_t *n_events, int64_t max_interval_ns,
                                uint64_t seed_lo, uint64_t n_seeds, uint32_t k, nmz_topk_entry *topk);
/* Waits for the plan's build and for the sweeps enqueued through it (not for the device or other streams). */
int nmz_replayable_plan_destroy(nmz_replayable_plan *plan);
/* Which statistics kernel the plan's sweeps take (diagnostic): 2 = wavelet-tree statistics (k_replayable_sweep_wt,
 * the default when 0 < max_interval < 2^32, the trace has <= 65,536 events -- a hint-length class of 4,096 or more
 * splits into sub-segments -- and the row image fits LDS),
 * 1 = order-query statistics (k_replayable_sweep_oq), 0 = per-decision sweeps; -1 for a NULL plan. The environment
 * variable NMZ_REPLAY_WT=0 at plan creation skips the wavelet trees (A/B runs). */
int nmz_replayable_plan_kernel(const nmz_replayable_plan *plan);
int nmz_replayable_sweep_dev(nmz_replayable_plan *plan, const uint32_t *d_seed_off,
                             const uint8_t *d_seed_bytes, uint64_t n_seeds,
                             nmz_sched_stats *d_stats, void *stream);
/* The same plus the top-k failure candidates (d_topk[k], k <= 256, by sum_delay desc then seed asc,
 * .seed = seed0 + seed index), enqueued in one call. Results equal nmz_replayable_sweep_dev +
 * nmz_topk_select_dev(seed0, k).
 * Same reference path as nmz_replayable_sweep (replayablepolicy.go:100-114); top-k is SURVEY A7. */
int nmz_replayable_sweep_topk_dev(nmz_replayable_plan *plan, const uint32_t *d_seed_off,
                                  const uint8_t *d_seed_bytes, uint64_t n_seeds, uint64_t seed0,
                                  uint32_t k, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk,
                                  void *stream);

/* The same sweep for the seeds "seed_lo", "seed_lo+1", ... "seed_lo+n_seeds-1": the decimal strings of those
 * uint64 integers (strconv.FormatUint, wrapping past 2^64), generated on the device, so a sweep over a range of
 * integer seeds needs no seed CSR in memory. Top-k .seed = the seed's integer value (seed_lo + index). Results
 * equal nmz_replayable_sweep_topk_dev over the CSR of those strings with seed0 = seed_lo. n_seeds <= max_seeds
 * of the plan. Same reference path (replayablepolicy.go:74-87 seed string, :100-114 interval). */
int nmz_replayable_sweep_decimal_topk_dev(nmz_replayable_plan *plan, uint64_t seed_lo, uint64_t n_seeds, uint32_t k,
                                          nmz_sched_stats *d_stats, nmz_topk_entry *d_topk, void *stream);

/* Online decisions (Replayable.QueueEvent -> determineInterval, replayablepolicy.go:100-126):
 * delays[e] = the interval of seed (seed_len bytes) for each of n_events pending events' hints
 * (CSR hint_off[n_events+1] into hint_bytes). No plan or tables: a batch of the events queued
 * since the last call, one thread per event. Synchronous; scratch is owned by the context. */
int nmz_replayable_decide(nmz_ctx *ctx, const uint8_t *seed, uint32_t seed_len, const uint32_t *hint_off,
                          const uint8_t *hint_bytes, uint32_t n_events, int64_t max_interval_ns, int64_t *delays);

/* ---- random policy sweep ------------------------------------------------
 * Seeds are the integers seed0 .. seed0+n_seeds-1. For seed s and event e
 * (evhash[e], evclass[e] = NMZ_EV_* bits) the decision is made by a fresh
 *     rng = rand.New(rand.NewSource(int64(FNV1a64(le64(s) || le64(evhash[e])))))
 * drawing, in this order,
 *     delay = rng.Int63n(max-min) + min   if min != max  (else delay = min, no draw)
 *     fault = rng.Intn(999) < fault_threshold            if NMZ_EV_FAULTABLE
 * with (min,max) = params->{min,max}_ns[prioritized].
 * Outputs (each may be NULL): stats[n_seeds]; delays/faults[n_dump_seeds*n_events];
 * topk[k] by (n_fault desc, sum_delay desc, seed asc), .seed = the seed value. */
int nmz_random_sweep(nmz_ctx *ctx, uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash,
                     const uint8_t *evclass, uint32_t n_events, const nmz_random_params *params,
                     nmz_sched_stats *stats, int64_t *delays, uint8_t *faults,
                     uint64_t n_dump_seeds, uint32_t k, nmz_topk_entry *topk);

/* Online decisions (Random.QueueEvent -> makeActionForEvent, randompolicy.go:300-346): the delay and
 * fault choice of one seed for each of n_events pending events, the same decision as
 * nmz_random_sweep makes for that seed and event. No plan; synchronous. */
int nmz_random_decide(nmz_ctx *ctx, uint64_t seed, const uint64_t *evhash, const uint8_t *evclass,
                      uint32_t n_events, const nmz_random_params *params, int64_t *delays, uint8_t *faults);

/* Device-resident variant: per-event tables are built once in the plan; the
 * sweep enqueues on `stream` and writes d_stats[n_seeds] (device memory). As for
 * replayable plans, one plan serves one stream at a time. */
typedef struct nmz_random_plan nmz_random_plan;
int nmz_random_plan_create(nmz_ctx *ctx, const uint64_t *evhash, const uint8_t *evclass,
                           uint32_t n_events, const nmz_random_params *params, uint64_t max_seeds,
                           nmz_random_plan **out);
int nmz_random_plan_destroy(nmz_random_plan *plan);
int nmz_random_sweep_dev(nmz_random_plan *plan, uint64_t seed0, uint64_t n_seeds,
                         nmz_sched_stats *d_stats, void *stream);

/* Top-k selection over device-resident stats (seed value = seed0 + index).
 * k <= 256 (here and for the sweeps' topk outputs); NMZ_EINVAL otherwise. */
int nmz_topk_select_dev(nmz_ctx *ctx, const nmz_sched_stats *d_stats, uint64_t n, uint64_t seed0,
                        uint32_t k, nmz_topk_entry *d_out, void *stream);
/* Merge n_lists top-k lists (d_lists[n_lists][k], each sorted as the sweeps write them: n_fault desc, sum_delay
 * desc, seed asc) into the best k (d_out[k]): the lists of several sweeps over disjoint seed ranges (successive
 * batches of one job, or the shards of one rank) become the job's top-k. d_lists and d_scratch (same size) are
 * overwritten. k <= 256. */
int nmz_topk_merge_dev(nmz_ctx *ctx, nmz_topk_entry *d_lists, uint64_t n_lists, uint32_t k,
                       nmz_topk_entry *d_scratch, nmz_topk_entry *d_out, void *stream);

/* ---- trace similarity (banded Levenshtein over event-hash sequences) ------
 * Traces in CSR: off[n_traces+1] (element offsets) into sym[] (uint64 event
 * hashes). ED_w(a,b) = min(D(n,m), w+1) where D is unit-cost Levenshtein
 * restricted to cells |i-j| <= w (cells outside the band are +inf).
 * ED_w == 0  <=>  the traces are equal element-wise (SingleTrace.Equals). */
int nmz_ed_pairs(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                 const uint32_t *pairs /* [2*n_pairs] */, uint64_t n_pairs, uint32_t band,
                 uint32_t *dist /* [n_pairs] */);

/* All pairs i != j; for each trace the k nearest others by (dist asc, id asc).
 * knn_id/knn_dist are [n_traces * k]; missing entries are NMZ_NONE. */
int nmz_ed_allpairs_knn(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym,
                        uint32_t n_traces, uint32_t band, uint32_t k, uint32_t *knn_id,
                        uint32_t *knn_dist);

/* Device-resident variant: the plan remaps symbols to dense ids and builds the
 * lane-interleaved candidate layout once; searches then run on resident data.
 * d_knn_keys[n_traces * k] (device) receives sorted keys (dist << 32 | id),
 * UINT64_MAX for missing entries. k in [1, 64]. */
typedef struct nmz_ed_plan nmz_ed_plan;
int nmz_ed_plan_create(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                       uint32_t band, nmz_ed_plan **out);
/* The same plan from event hashes already in device memory: off (host, n_traces + 1 offsets) and d_sym (device,
 * off[n_traces] u64, read during the call). Multi-GPU callers upload 1/N of the symbols per device and all_gather
 * them over RCCL instead of pushing the whole store through every device's PCIe link. */
int nmz_ed_plan_create_dev(nmz_ctx *ctx, const uint64_t *off, const uint64_t *d_sym, uint32_t n_traces,
                           uint32_t band, nmz_ed_plan **out);
/* Plan options (bit flags) of nmz_ed_plan_create_opts. 0 is the product's choice; the others select the
 * alternative forms of the bit-parallel search, for A/B runs and tests. Whichever form a plan takes, a shard owns
 * the same pairs (whole 64-query blocks, nmz_ed_block_shard), so within ONE process the shards of a search may run on
 * plans of different forms and still partition the pairs (tests/test_ed_gpu.py checks this). The multi-rank paths do
 * not allow the mix: the device groups and namazu_amd/dist.check_ed_plans require equal fingerprints, which include
 * the form bits, and fail with NMZ_EINVAL otherwise. The NMZ_ED_* environment knobs that add to these are read only
 * when NMZ_AB=1 is set. */
#define NMZ_ED_OPT_SINGLE_KERNEL 1u /* no two-phase search: the single kernel with its in-workgroup pre-filter */
#define NMZ_ED_OPT_NO_QGRAM 2u      /* no q-gram lower-bound filter (the single kernel, without the filter) */
#define NMZ_ED_OPT_COMPACT 4u       /* compact per-workgroup Peq tables even when the direct tables fit */
#define NMZ_ED_OPT_HOST_BUILD 8u    /* the plan's streams built on the host instead of the device */
/* sym (host) or d_sym (device, read during the call): exactly one of them when the store is not empty */
int nmz_ed_plan_create_opts(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint64_t *d_sym,
                            uint32_t n_traces, uint32_t band, uint32_t opts, nmz_ed_plan **out);
/* The plan's fingerprint, 8 words: version, kernel kind | band << 8 | template band << 40, n_traces, total
 * symbols, two-phase | q-gram << 1 | compact << 2, block-row queries | pool << 32, FNV-1a 64 of the offsets, alphabet
 * size. Ranks that search one store together must hold equal fingerprints: the device groups all_gather them when
 * a plan is created and fail with NMZ_EINVAL when they differ. */
#define NMZ_ED_FP_WORDS 8
#define NMZ_ED_FP_VERSION 1u
int nmz_ed_plan_fingerprint(const nmz_ed_plan *plan, uint64_t *fp /* [NMZ_ED_FP_WORDS] */);
int nmz_ed_plan_destroy(nmz_ed_plan *plan);
int nmz_ed_plan_is_fast(const nmz_ed_plan *plan);
int nmz_ed_allpairs_knn_dev(nmz_ed_plan *plan, uint32_t k, uint64_t *d_knn_keys, void *stream);
/* Multi-GPU: shard `shard` of `n_shards` processes every n_shards-th work chunk;
 * its keys are partial lists. nmz_knn_merge_dev merges n_parts partial lists
 * ([n_parts][n_traces][k], e.g. after an RCCL all_gather), and nmz_ed_knn_fill_dev
 * then completes the merged lists: on a bit-parallel plan (nmz_ed_plan_is_fast == 2) a
 * shard lists only its pairs within the band, and every other pair's result is band + 1,
 * so the merged lists take (band + 1, id) for the smallest ids not listed (not the trace
 * itself), in increasing id, up to k. On other plans the fill leaves complete lists
 * unchanged. (nmz_ed_allpairs_knn[_dev] fill by themselves.) */
/* Host-only (no device work): the shard that owns query block qb (queries 64 qb .. 64 qb + 63) of the
 * bit-parallel search (both forms: two-phase and the single kernel) under nmz_ed_allpairs_knn_shard_dev with n_shards shards: every pair (i, j), i < j, belongs
 * to the shard of block i / 64, in rotated snake order (in each period of 2 n_shards blocks, block r and its mirror
 * 2 n_shards - 1 - r form pair p = min(r, 2 n_shards - 1 - r), which goes to shard (p + period) mod n_shards). A
 * fixed rule, the same in every process (no environment knob). A shard whose entry lists exceed the two-phase limit
 * runs its own query blocks in batches, so every shard of a search deals by this rule. tests/test_dist_cpu.py deals
 * pairs by it. */
uint32_t nmz_ed_block_shard(uint32_t qb, uint32_t n_shards);
int nmz_ed_allpairs_knn_shard_dev(nmz_ed_plan *plan, uint32_t k, uint32_t shard, uint32_t n_shards,
                                  uint64_t *d_knn_keys, void *stream);
int nmz_knn_merge_dev(nmz_ctx *ctx, const uint64_t *d_parts, uint32_t n_parts, uint32_t n_traces,
                      uint32_t k, uint64_t *d_out, void *stream);
int nmz_ed_knn_fill_dev(nmz_ed_plan *plan, uint32_t k, uint64_t *d_knn_keys, void *stream);
/* Single queries against a resident store (HistoryStorage similarity search; the reference's own
 * search re-decodes every stored trace per query, naive.go:235-252 "FIXME: quite ineffective"):
 * the plan's stored traces stay on the device; each of n_queries query traces (CSR q_off/q_sym,
 * u64 event hashes, any length) gets its k nearest stored traces by (ED_band asc, id asc), ED_band
 * as in nmz_ed_pairs. knn_id/knn_dist are [n_queries * k], NMZ_NONE where fewer than k traces
 * exist. Any plan and band: bit-parallel plans (band <= 64) run k_ed_bv's query form, wide plans
 * (64 < band <= 8,192) k_ed_wide_query, the others (and queries longer than the plan's kernel
 * takes) a generic per-pair kernel over the resident store. 1 <= k <= 64. Synchronous. */
int nmz_ed_plan_query_knn(nmz_ed_plan *plan, const uint64_t *q_off, const uint64_t *q_sym, uint32_t n_queries,
                          uint32_t k, uint32_t *knn_id, uint32_t *knn_dist);
/* Work counters of the plan's latest search (synchronises `stream`, NULL = the context's stream).
 * out[NMZ_ED_NCOUNTERS]: the bit-parallel band kernel (nmz_ed_plan_is_fast == 2) fills
 *   [0] pairs that ran the DP, [1] pairs whose result is <= band (in band),
 *   [2] candidate x 32-column blocks executed (each block steps 2 query columns per candidate),
 *   [3] candidates that ran the DP, [4] live query-blocks (blocks x queries still running),
 *   [5] pairs inside the length band whose result the q-gram lower bound settled at band + 1
 *       without a DP;
 * other kernels keep no counters and leave zeros. Diagnostics for the bench, not part of the
 * reference interface. */
#define NMZ_ED_NCOUNTERS 6
int nmz_ed_plan_counters(nmz_ed_plan *plan, uint64_t *out, void *stream);
/* Test hook, not part of the reference interface: the two-phase search's offset kernels (k_tp_reduce, k_tp_scan)
 * on caller data. d_cnt[n] (device) -> d_poff[n + 1] = exclusive prefix sums of the counts mod 2^32,
 * d_ioff[n + 1] = exclusive prefix sums of ceil(count / item) mod 2^32, *d_tot = the 64-bit count total;
 * item a power of two. Enqueued on `stream` (NULL = the context's stream), synchronised before it returns. */
int nmz_debug_tp_offsets(nmz_ctx *ctx, const uint32_t *d_cnt, uint32_t n, uint32_t item, uint32_t *d_poff,
                         uint32_t *d_ioff, uint64_t *d_tot, void *stream);

/* ---- trace equality classes (nmz tools visualize) ------------------------
 * Replaces the O(n^2) loops of cli/tools/visualize.go:51-172 (gnuplot): trace i is a
 * repeat iff an earlier trace equals it.
 *   entity == NULL: exact mode (seenBefore, :51-60) -- sequence equality of sym[], i.e.
 *       SingleTrace.Equals / AreActionsSliceEqual (util/signal/misc.go:22-35) when sym[] are
 *       action symbols (namazu_amd/historystorage.py).
 *   entity != NULL: partial-order mode, the reference default (-po-reduction=true, :42;
 *       createTracesPerEntity / tracesEqualInPO :62-124): entity[t] is the element's entity
 *       id, dense per trace (< 16384), NMZ_NONE for actions without an event (skipped);
 *       sym[] are event symbols (Event.Equals). Traces are equal iff every entity's projected
 *       subsequence is equal.
 * sig[2*n_traces]: 128-bit signature per trace (equal traces -> equal signatures; distinct
 * ones collide with probability ~2^-128). first_equal[i] = the smallest j with sig_j == sig_i
 * (j <= i), so the unique-trace curve of visualize is the running count of first_equal[i] == i. */
int nmz_trace_signatures(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint32_t *entity,
                         uint32_t n_traces, uint64_t *sig);
int nmz_unique_traces(nmz_ctx *ctx, const uint64_t *off, const uint64_t *sym, const uint32_t *entity,
                      uint32_t n_traces, uint32_t *first_equal);
/* Device-resident variant: d_entity may be NULL (exact mode); entity ids must be < max_entities (<= 16384;
 * larger ids are skipped like NMZ_NONE, so the caller must pass the true bound);
 * d_sig[2*n_traces] receives the signatures. Enqueued on `stream` (NULL = the context's). */
int nmz_unique_traces_dev(nmz_ctx *ctx, const uint64_t *d_off, const uint64_t *d_sym, const uint32_t *d_entity,
                          uint32_t n_traces, uint32_t max_entities, uint64_t *d_sig, uint32_t *d_first_equal,
                          void *stream);

/* ---- device groups: several GPUs behind one call (multi-GPU inside the C ABI) ----------------------------
 * The reference's callers are single processes (cli/run.go:123-136 initPolicy; cli/tools/visualize.go:138-172),
 * so one process must reach every GPU of a node. A group holds one context and one worker thread per device
 * (bound to its device once, so a cgo caller may call from any OS thread) and one RCCL communicator over the
 * devices, created once. Work is cut into n_shards shards (0 = one per rank; more than the ranks = "virtual"
 * shards, so a single GPU runs the sharding and merge logic of any shard count); shard s runs on rank
 * s mod n_ranks. Sweeps shard by contiguous seed range (sizes differ by <= 1), the all-pairs search by the
 * plan's query-block deal (rotated snake order, nmz_ed_block_shard). Each rank merges its shards on its device,
 * one RCCL
 * all_gather over xGMI exchanges the ranks' lists, and a deterministic merge -- (n_fault desc, sum_delay desc,
 * seed asc) for top-k, (dist asc, id asc) for k-NN -- makes the result identical to one unsharded call.
 * Group calls are synchronous and serialised per group; host buffers are borrowed for the call only. A group call
 * never changes the calling thread's current HIP device (nor does any single-context call). */
typedef struct nmz_group nmz_group;
#define NMZ_GROUP_ID_BYTES 128
/* bit d of dev_mask = device d */
int nmz_open_group(uint32_t dev_mask, uint32_t n_shards, nmz_group **out);
/* One process per device (several hosts, or a launcher with a process per GPU): rank 0 makes the id
 * (nmz_group_unique_id) and hands it to every rank out of band; each rank opens its device. Every rank receives
 * the merged results. stats outputs hold the seeds of this rank's shards only. */
int nmz_group_unique_id(uint8_t *id /* [NMZ_GROUP_ID_BYTES] */);
int nmz_open_group_rank(const uint8_t *id, int n_ranks, int rank, int device, uint32_t n_shards, nmz_group **out);
/* Waits for a group call already in progress, then frees the group; NMZ_EINVAL while group plans made on it are
 * still alive (destroy them first). No call on the group may start once close has begun. */
int nmz_close_group(nmz_group *g);
int nmz_group_info(const nmz_group *g, int *n_ranks, int *n_local_devices, uint32_t *n_shards);
/* Collectives this process has entered on the group so far. Every group call that exchanges results first enters
 * one status all_gather (every rank, whatever failed locally) and then, only when every rank succeeded, its payload
 * collective, so a failed call enters the same collectives on every rank (tests check the sequence with this). */
int nmz_group_collectives(const nmz_group *g, uint64_t *n);

/* replayable sweep over a group (replayablepolicy.go:100-114 per decision, as nmz_replayable_sweep): one plan
 * per device, kept for repeated sweeps; stats[n_seeds] (may be NULL) and the merged topk[k] (k <= 256, .seed =
 * seed index, or the seed's integer value for the decimal form) go to host memory. */
typedef struct nmz_replayable_group_plan nmz_replayable_group_plan;
int nmz_replayable_group_plan_create(nmz_group *g, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                     uint32_t n_events, int64_t max_interval_ns, uint64_t max_seeds_per_shard,
                                     nmz_replayable_group_plan **out);
int nmz_replayable_group_plan_destroy(nmz_replayable_group_plan *gp);
int nmz_replayable_group_sweep(nmz_replayable_group_plan *gp, const uint32_t *seed_off, const uint8_t *seed_bytes,
                               uint64_t n_seeds, uint32_t k, nmz_sched_stats *stats, nmz_topk_entry *topk);
/* seeds = decimal strings of seed_lo .. seed_lo + n_seeds - 1 (nmz_replayable_sweep_decimal_topk_dev) */
int nmz_replayable_group_sweep_decimal(nmz_replayable_group_plan *gp, uint64_t seed_lo, uint64_t n_seeds, uint32_t k,
                                       nmz_sched_stats *stats, nmz_topk_entry *topk);
/* one call: plan + sweep + merged top-k (the group form of nmz_replayable_sweep) */
int nmz_replayable_sweep_topk_group(nmz_group *g, const uint32_t *seed_off, const uint8_t *seed_bytes,
                                    uint64_t n_seeds, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                    uint32_t n_events, int64_t max_interval_ns, uint32_t k, nmz_sched_stats *stats,
                                    nmz_topk_entry *topk);

/* random-policy sweep over a group (randompolicy.go:300-346, as nmz_random_sweep): seeds seed0 .. seed0+n-1. */
typedef struct nmz_random_group_plan nmz_random_group_plan;
int nmz_random_group_plan_create(nmz_group *g, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                                 const nmz_random_params *params, uint64_t max_seeds_per_shard,
                                 nmz_random_group_plan **out);
int nmz_random_group_plan_destroy(nmz_random_group_plan *gp);
int nmz_random_group_sweep(nmz_random_group_plan *gp, uint64_t seed0, uint64_t n_seeds, uint32_t k,
                           nmz_sched_stats *stats, nmz_topk_entry *topk);
int nmz_random_sweep_topk_group(nmz_group *g, uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash,
                                const uint8_t *evclass, uint32_t n_events, const nmz_random_params *params,
                                uint32_t k, nmz_sched_stats *stats, nmz_topk_entry *topk);

/* all-pairs banded edit-distance k-NN over a group (as nmz_ed_allpairs_knn): every device holds the store. The
 * store reaches the devices as 1/n_ranks shares: rank r uploads symbols [r S, r S + S) (S = ceil(total / n_ranks))
 * through its own PCIe link, one RCCL all_gather over xGMI assembles the store on every device, and each device
 * builds its plan from device memory (nmz_ed_plan_create_dev). nmz_ed_group_plan_timing reports, per local device,
 * the share upload, the all_gather and the device plan build (ms, arrays of nmz_group_info's n_local_devices).
 * After each local step (upload, plan build) the ranks exchange their status, so a rank that failed never leaves the
 * others waiting in a collective; after the build they exchange their plans' fingerprints (nmz_ed_plan_fingerprint)
 * and all fail with NMZ_EINVAL when any two differ. */
typedef struct nmz_ed_group_plan nmz_ed_group_plan;
int nmz_ed_group_plan_create(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                             uint32_t band, nmz_ed_group_plan **out);
/* The same with NMZ_ED_OPT_* plan options for every member's plan (nmz_ed_plan_create_opts). */
int nmz_ed_group_plan_create_opts(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                                  uint32_t band, uint32_t opts, nmz_ed_group_plan **out);
int nmz_ed_group_plan_timing(const nmz_ed_group_plan *gp, double *upload_ms, double *gather_ms, double *build_ms);
int nmz_ed_group_plan_destroy(nmz_ed_group_plan *gp);
int nmz_ed_group_allpairs_knn(nmz_ed_group_plan *gp, uint32_t k, uint32_t *knn_id, uint32_t *knn_dist);
int nmz_ed_allpairs_knn_group(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                              uint32_t band, uint32_t k, uint32_t *knn_id, uint32_t *knn_dist);

#ifdef __cplusplus
}
#endif
#endif /* NMZ_GPU_H */
