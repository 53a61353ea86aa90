/*
 * nmz_oracle.c -- CPU ORACLE (test infrastructure only).
 *
 * Plain-C restatement of the reference's decision and trace-comparison
 * semantics, used ONLY by tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg as the checker. Nothing in the product (namazu_amd/)
 * links, loads or calls this file.
 *
 * It deliberately follows the reference's naive per-event algorithm (fresh
 * FNV hasher per decision, full Go rngSource seeding per decision) rather
 * than the product's algebraic shortcuts, so the two are independent.
 *
 * Pinning: the reference is Go (no toolchain here, and the arithmetic lives
 * in the un-vendored Go 1.10 standard library), so it is not compiled. The
 * primitives are pinned by published known-answer vectors (FNV-1a 64 test
 * vectors; Go math/rand seed-1 outputs) in tests/test_oracle.py. The policy
 * compositions (replayable, random) follow the cited reference lines; the
 * reference's tests assert no numeric values for them, so at
 * that level parity is "unpinned" beyond the KATs.
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "../include/nmz_gpu.h"

#ifdef _OPENMP
#include <omp.h>
#endif

/* ---------------------------------------------------------------------- */
/* hash/fnv New64a (Go 1.10 src/hash/fnv/fnv.go)                           */
/* ---------------------------------------------------------------------- */
#define FNV64_OFFSET 0xcbf29ce484222325ULL
#define FNV64_PRIME 0x100000001b3ULL

uint64_t nmzo_fnv1a64_update(uint64_t h, const uint8_t *p, size_t n) {
    for (size_t i = 0; i < n; i++) {
        h ^= (uint64_t)p[i];
        h *= FNV64_PRIME;
    }
    return h;
}

uint64_t nmzo_fnv1a64(const uint8_t *p, size_t n) { return nmzo_fnv1a64_update(FNV64_OFFSET, p, n); }

/* ---------------------------------------------------------------------- */
/* Go math/rand rngSource (Go 1.10 src/math/rand/rng.go, rand.go)           */
/* ---------------------------------------------------------------------- */
#define RNG_LEN 607
#define RNG_TAP 273
#define INT32MAX 2147483647LL
#define MASK63 0x7fffffffffffffffULL

static uint64_t g_cooked[RNG_LEN];
static int g_cooked_ready = 0;

static int32_t seedrand(int32_t x) {
    /* seed rng x[n+1] = 48271 * x[n] mod (2**31 - 1), Schrage form */
    const int32_t A = 48271, Q = 44488, R = 3399;
    int32_t hi = x / Q, lo = x % Q;
    x = A * lo - R * hi;
    if (x < 0) x += (int32_t)INT32MAX;
    return x;
}

/* r = a*b mod (x^607 - x^334 - 1) over Z/2^64 */
static void polymulmod(const uint64_t *a, const uint64_t *b, uint64_t *r) {
    uint64_t t[2 * RNG_LEN];
    memset(t, 0, sizeof t);
    for (int i = 0; i < RNG_LEN; i++)
        for (int j = 0; j < RNG_LEN; j++) t[i + j] += a[i] * b[j];
    for (int k = 2 * RNG_LEN - 2; k >= RNG_LEN; k--) {
        t[k - RNG_LEN + 334] += t[k];
        t[k - RNG_LEN] += t[k];
        t[k] = 0;
    }
    memcpy(r, t, RNG_LEN * sizeof(uint64_t));
}

/* Derive rngCooked from first principles (gen_cooked.go): srand(1) with
 * 20/10-bit shifts, then 7.8e12 additive-LFG steps, by jump-ahead. */
static void derive_cooked(void) {
    uint64_t vec0[RNG_LEN];
    int32_t x = 1;
    for (int i = -20; i < RNG_LEN; i++) {
        x = seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 20;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x << 10;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            vec0[i] = u;
        }
    }
    /* output y_s lives at position (333 - s) mod 607; z_k = y_{k-607} */
    uint64_t z[2 * RNG_LEN];
    for (int k = 0; k < RNG_LEN; k++) z[k] = vec0[((333 - (k - RNG_LEN)) % RNG_LEN + RNG_LEN) % RNG_LEN];
    for (int k = RNG_LEN; k < 2 * RNG_LEN - 1; k++) z[k] = z[k - RNG_LEN] + z[k - RNG_TAP];
    const uint64_t N = 7800000000000ULL;
    uint64_t r[RNG_LEN] = {1}, base[RNG_LEN] = {0, 1}, tmp[RNG_LEN];
    for (uint64_t e = N; e; e >>= 1) {
        if (e & 1) { polymulmod(r, base, tmp); memcpy(r, tmp, sizeof r); }
        if (e >> 1) { polymulmod(base, base, tmp); memcpy(base, tmp, sizeof base); }
    }
    for (int j = 0; j < RNG_LEN; j++) {
        uint64_t acc = 0;
        for (int i = 0; i < RNG_LEN; i++) acc += r[i] * z[i + j];
        uint64_t t = N - RNG_LEN + (uint64_t)j;
        g_cooked[(333 + 20000000000ULL * RNG_LEN - t) % RNG_LEN] = acc;
    }
    g_cooked_ready = 1;
}

void nmzo_init(void) {
    if (!g_cooked_ready) derive_cooked();
}

void nmzo_go_rng_cooked(int64_t *out) {
    nmzo_init();
    for (int i = 0; i < RNG_LEN; i++) out[i] = (int64_t)g_cooked[i];
}

typedef struct nmzo_go_rng {
    int tap, feed;
    int64_t n_out; /* outputs drawn since Seed (diagnostic) */
    uint64_t vec[RNG_LEN];
} nmzo_go_rng;

/* rngSource.Seed (rng.go) */
void nmzo_go_seed(nmzo_go_rng *rng, int64_t seed) {
    rng->tap = 0;
    rng->feed = RNG_LEN - RNG_TAP;
    rng->n_out = 0;
    seed = seed % INT32MAX;
    if (seed < 0) seed += INT32MAX;
    if (seed == 0) seed = 89482311;
    int32_t x = (int32_t)seed;
    for (int i = -20; i < RNG_LEN; i++) {
        x = seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << 40;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x << 20;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            u ^= g_cooked[i];
            rng->vec[i] = u;
        }
    }
}

uint64_t nmzo_go_uint64(nmzo_go_rng *rng) {
    rng->tap--;
    if (rng->tap < 0) rng->tap += RNG_LEN;
    rng->feed--;
    if (rng->feed < 0) rng->feed += RNG_LEN;
    uint64_t x = rng->vec[rng->feed] + rng->vec[rng->tap];
    rng->vec[rng->feed] = x;
    rng->n_out++;
    return x;
}

int64_t nmzo_go_int63(nmzo_go_rng *rng) { return (int64_t)(nmzo_go_uint64(rng) & MASK63); }
int32_t nmzo_go_int31(nmzo_go_rng *rng) { return (int32_t)(nmzo_go_int63(rng) >> 32); }

/* Rand.Int63n (rand.go); n > 0 */
int64_t nmzo_go_int63n(nmzo_go_rng *rng, int64_t n) {
    if (n <= 0) return -1;
    if ((n & (n - 1)) == 0) return nmzo_go_int63(rng) & (n - 1);
    int64_t max = (int64_t)((1ULL << 63) - 1 - (1ULL << 63) % (uint64_t)n);
    int64_t v = nmzo_go_int63(rng);
    while (v > max) v = nmzo_go_int63(rng);
    return v % n;
}

/* Rand.Int31n (rand.go); n > 0 */
int32_t nmzo_go_int31n(nmzo_go_rng *rng, int32_t n) {
    if (n <= 0) return -1;
    if ((n & (n - 1)) == 0) return nmzo_go_int31(rng) & (n - 1);
    int32_t max = (int32_t)((1U << 31) - 1 - (1U << 31) % (uint32_t)n);
    int32_t v = nmzo_go_int31(rng);
    while (v > max) v = nmzo_go_int31(rng);
    return v % n;
}

/* Rand.Intn (rand.go): Int31n for n <= 2^31-1 */
int64_t nmzo_go_intn(nmzo_go_rng *rng, int64_t n) {
    if (n <= 0) return -1;
    if (n <= INT32MAX) return nmzo_go_int31n(rng, (int32_t)n);
    return nmzo_go_int63n(rng, n);
}

/* ---------------------------------------------------------------------- */
/* statistics helpers (A7)                                                 */
/* ---------------------------------------------------------------------- */
static void stats_init(nmz_sched_stats *s) {
    s->sum_delay_ns = 0;
    s->max_delay_ns = INT64_MIN;
    s->argmax_event = NMZ_NONE;
    s->n_fault = 0;
    s->first_fault = NMZ_NONE;
    s->flags = 0;
}

static void stats_add(nmz_sched_stats *s, uint32_t e, int64_t delay, int fault) {
    s->sum_delay_ns += (uint64_t)delay;
    if (s->argmax_event == NMZ_NONE || delay > s->max_delay_ns) {
        s->max_delay_ns = delay;
        s->argmax_event = e;
    }
    if (fault) {
        if (s->first_fault == NMZ_NONE) s->first_fault = e;
        s->n_fault++;
    }
}

/* ---------------------------------------------------------------------- */
/* replayable policy: replayablepolicy.go:100-114                          */
/* ---------------------------------------------------------------------- */
int64_t nmzo_replayable_interval(const uint8_t *seed, size_t seed_len, const uint8_t *hint,
                                 size_t hint_len, int64_t max_interval) {
    if (max_interval == 0) return 0; /* :101-104 */
    uint64_t h = FNV64_OFFSET;       /* :106 fnv.New64a() */
    h = nmzo_fnv1a64_update(h, seed, seed_len); /* :107 h.Write([]byte(r.Seed)) */
    h = nmzo_fnv1a64_update(h, hint, hint_len); /* :108 h.Write([]byte(hint)) */
    return (int64_t)(h % (uint64_t)max_interval); /* :110 */
}

void nmzo_replayable_sweep(const uint32_t *seed_off, const uint8_t *seed_bytes, uint64_t n_seeds,
                           const uint32_t *hint_off, const uint8_t *hint_bytes, uint32_t n_events,
                           int64_t max_interval, nmz_sched_stats *stats, int64_t *delays,
                           uint64_t n_dump, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 64)
#endif
    for (int64_t s = 0; s < (int64_t)n_seeds; s++) {
        nmz_sched_stats st;
        stats_init(&st);
        const uint8_t *sp = seed_bytes + seed_off[s];
        size_t sl = seed_off[s + 1] - seed_off[s];
        for (uint32_t e = 0; e < n_events; e++) {
            int64_t t = nmzo_replayable_interval(sp, sl, hint_bytes + hint_off[e],
                                                 hint_off[e + 1] - hint_off[e], max_interval);
            stats_add(&st, e, t, 0);
            if (delays && (uint64_t)s < n_dump) delays[(uint64_t)s * n_events + e] = t;
        }
        if (stats) stats[s] = st;
    }
}

/* ---------------------------------------------------------------------- */
/* random policy: randompolicy.go:300-316,332-346 + util/queue/impl.go      */
/* ---------------------------------------------------------------------- */

/* LoadConfig/QueueEvent parameter semantics (randompolicy.go:223-225,337-339,
 * queue/impl.go:36-38). Returns 0 or NMZ_EINVAL. */
int nmzo_random_params(int64_t min_ns, int64_t max_ns, double p, nmz_random_params *out) {
    if (p < 0.0 || p > 1.0 || p != p) return NMZ_EINVAL;
    out->min_ns[0] = min_ns;
    out->max_ns[0] = max_ns;
    out->min_ns[1] = (int64_t)((double)min_ns * 0.8);
    out->max_ns[1] = (int64_t)((double)max_ns * 0.8);
    out->fault_threshold = (int32_t)(p * 1000.0);
    out->reserved = 0;
    if (out->min_ns[0] > out->max_ns[0] || out->min_ns[1] > out->max_ns[1]) return NMZ_EINVAL;
    return 0;
}

/* per-event seed of the deterministic restatement: FNV1a64(le64(seed) || le64(evhash)) */
int64_t nmzo_random_event_seed(uint64_t seed, uint64_t evhash) {
    uint8_t buf[16];
    for (int i = 0; i < 8; i++) {
        buf[i] = (uint8_t)(seed >> (8 * i));
        buf[8 + i] = (uint8_t)(evhash >> (8 * i));
    }
    return (int64_t)nmzo_fnv1a64(buf, 16);
}

/* One decision. Returns the number of Go rng outputs consumed. */
int nmzo_random_decide(uint64_t seed, uint64_t evhash, uint8_t evclass, const nmz_random_params *p,
                       int64_t *delay, int *fault) {
    nmzo_go_rng rng;
    nmzo_go_seed(&rng, nmzo_random_event_seed(seed, evhash));
    int pr = (evclass & NMZ_EV_PRIORITIZED) ? 1 : 0;
    int64_t mn = p->min_ns[pr], mx = p->max_ns[pr];
    if (mn == mx) {
        *delay = mn; /* fixed-duration FIFO path, no draw (impl.go:117-119) */
    } else {
        *delay = nmzo_go_int63n(&rng, mx - mn) + mn; /* determineDuration, impl.go:95-97 */
    }
    *fault = 0;
    if (evclass & NMZ_EV_FAULTABLE) /* randompolicy.go:307-310 */
        *fault = nmzo_go_intn(&rng, 999) < (int64_t)p->fault_threshold;
    return (int)rng.n_out;
}

static int topk_better(const nmz_topk_entry *a, const nmz_topk_entry *b) {
    if (a->n_fault != b->n_fault) return a->n_fault > b->n_fault;
    if (a->sum_delay_ns != b->sum_delay_ns) return a->sum_delay_ns > b->sum_delay_ns;
    return a->seed < b->seed;
}

/* insert into a sorted top-k list of current length *n (capacity k) */
static void topk_insert(nmz_topk_entry *list, uint32_t *n, uint32_t k, const nmz_topk_entry *x) {
    if (k == 0) return;
    if (*n == k && !topk_better(x, &list[k - 1])) return;
    uint32_t pos = (*n < k) ? (*n)++ : k - 1;
    while (pos > 0 && topk_better(x, &list[pos - 1])) {
        list[pos] = list[pos - 1];
        pos--;
    }
    list[pos] = *x;
}

/* Top-k over a stats array. seed value of entry i is seed0 + i. */
void nmzo_topk_from_stats(const nmz_sched_stats *stats, uint64_t n, uint64_t seed0, uint32_t k,
                          nmz_topk_entry *out) {
    uint32_t cnt = 0;
    for (uint64_t i = 0; i < n; i++) {
        nmz_topk_entry x = {seed0 + i, (int64_t)stats[i].sum_delay_ns, stats[i].n_fault,
                            stats[i].first_fault};
        topk_insert(out, &cnt, k, &x);
    }
    for (uint32_t i = cnt; i < k; i++) {
        out[i].seed = UINT64_MAX;
        out[i].sum_delay_ns = INT64_MIN;
        out[i].n_fault = 0;
        out[i].first_fault = NMZ_NONE;
    }
}

void nmzo_random_sweep(uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash, const uint8_t *evclass,
                       uint32_t n_events, const nmz_random_params *p, nmz_sched_stats *stats,
                       int64_t *delays, uint8_t *faults, uint64_t n_dump, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t s = 0; s < (int64_t)n_seeds; s++) {
        nmz_sched_stats st;
        stats_init(&st);
        for (uint32_t e = 0; e < n_events; e++) {
            int64_t d;
            int f;
            nmzo_random_decide(seed0 + (uint64_t)s, evhash[e], evclass[e], p, &d, &f);
            stats_add(&st, e, d, f);
            if ((uint64_t)s < n_dump) {
                if (delays) delays[(uint64_t)s * n_events + e] = d;
                if (faults) faults[(uint64_t)s * n_events + e] = (uint8_t)f;
            }
        }
        if (stats) stats[s] = st;
    }
}

/* ---------------------------------------------------------------------- */
/* trace distance (build-defined extension; distance 0 <=> Equals,         */
/* util/trace/trace.go:29-31, util/signal/misc.go:22-35)                   */
/* ---------------------------------------------------------------------- */

/* full unit-cost Levenshtein, O(n*m) */
uint64_t nmzo_levenshtein(const uint64_t *a, uint64_t n, const uint64_t *b, uint64_t m) {
    uint64_t *row = (uint64_t *)malloc((m + 1) * sizeof(uint64_t));
    for (uint64_t j = 0; j <= m; j++) row[j] = j;
    for (uint64_t i = 1; i <= n; i++) {
        uint64_t diag = row[0];
        row[0] = i;
        for (uint64_t j = 1; j <= m; j++) {
            uint64_t up = row[j];
            uint64_t v = diag + (a[i - 1] != b[j - 1]);
            if (up + 1 < v) v = up + 1;
            if (row[j - 1] + 1 < v) v = row[j - 1] + 1;
            row[j] = v;
            diag = up;
        }
    }
    uint64_t d = row[m];
    free(row);
    return d;
}

/* banded: min(D_band(n,m), w+1), cells with |i-j| > w are +inf */
uint32_t nmzo_levenshtein_banded(const uint64_t *a, uint64_t n, const uint64_t *b, uint64_t m,
                                 uint32_t w) {
    const uint64_t INF = UINT64_MAX / 4;
    uint64_t diff = n > m ? n - m : m - n;
    if (diff > w) return w + 1;
    uint64_t *row = (uint64_t *)malloc((m + 1) * sizeof(uint64_t));
    for (uint64_t j = 0; j <= m; j++) row[j] = (j <= w) ? j : INF;
    for (uint64_t i = 1; i <= n; i++) {
        uint64_t jlo = (i > w) ? i - w : 0, jhi = (i + w < m) ? i + w : m;
        /* row holds D[i-1][*]; compute D[i][jlo..jhi] in place */
        uint64_t diag = (jlo > 0) ? row[jlo - 1] : INF; /* D[i-1][jlo-1] */
        uint64_t left = INF;                           /* D[i][jlo-1]: out of band */
        if (jlo == 0) {
            diag = INF;
            left = INF;
        }
        for (uint64_t j = jlo; j <= jhi; j++) {
            uint64_t up = row[j]; /* D[i-1][j] (INF if it was out of band) */
            uint64_t v;
            if (j == 0) {
                v = i; /* D[i][0] = i, in band since i <= w here */
            } else {
                v = diag + (a[i - 1] != b[j - 1]);
                if (up + 1 < v) v = up + 1;
                if (left + 1 < v) v = left + 1;
            }
            if (v > INF) v = INF;
            row[j] = v;
            diag = up;
            left = v;
        }
        if (jlo > 0) row[jlo - 1] = INF; /* D[i][jlo-1] is out of band */
    }
    uint64_t d = row[m];
    free(row);
    return d > w ? w + 1 : (uint32_t)d;
}

void nmzo_ed_pairs(const uint64_t *off, const uint64_t *sym, const uint32_t *pairs, uint64_t n_pairs,
                   uint32_t w, uint32_t *dist, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 16)
#endif
    for (int64_t p = 0; p < (int64_t)n_pairs; p++) {
        uint32_t i = pairs[2 * p], j = pairs[2 * p + 1];
        dist[p] = nmzo_levenshtein_banded(sym + off[i], off[i + 1] - off[i], sym + off[j],
                                          off[j + 1] - off[j], w);
    }
}

/* brute-force all-pairs kNN: (dist asc, id asc), self excluded */
void nmzo_ed_allpairs_knn(const uint64_t *off, const uint64_t *sym, uint32_t n, uint32_t w, uint32_t k,
                          uint32_t *knn_id, uint32_t *knn_dist, int nthreads) {
#ifdef _OPENMP
    if (nthreads > 0) omp_set_num_threads(nthreads);
#pragma omp parallel for schedule(dynamic, 1)
#endif
    for (int64_t q = 0; q < (int64_t)n; q++) {
        uint32_t *ids = knn_id + (uint64_t)q * k, *ds = knn_dist + (uint64_t)q * k;
        uint32_t cnt = 0;
        for (uint32_t c = 0; c < n; c++) {
            if (c == (uint32_t)q) continue;
            uint32_t d = nmzo_levenshtein_banded(sym + off[q], off[q + 1] - off[q], sym + off[c],
                                                 off[c + 1] - off[c], w);
            if (k == 0) continue;
            if (cnt == k && d >= ds[k - 1]) continue; /* ids ascend, so ties lose */
            uint32_t pos = (cnt < k) ? cnt++ : k - 1;
            while (pos > 0 && d < ds[pos - 1]) {
                ds[pos] = ds[pos - 1];
                ids[pos] = ids[pos - 1];
                pos--;
            }
            ds[pos] = d;
            ids[pos] = c;
        }
        for (uint32_t i = cnt; i < k; i++) {
            ids[i] = NMZ_NONE;
            ds[i] = NMZ_NONE;
        }
    }
}
