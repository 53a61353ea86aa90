/* The C oracle (test infrastructure) under ASan + UBSan: every entry point on edge inputs (empty traces, band 0,
 * bands wider than the traces, rejection-heavy Int63n spans, wrapped seed ranges, k larger than n). Exit 0 = clean. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "../../include/nmz_gpu.h"

typedef struct nmzo_go_rng {
    int tap, feed;
    int64_t n_out;
    uint64_t vec[607];
} nmzo_go_rng;
void nmzo_init(void);
uint64_t nmzo_fnv1a64(const uint8_t *p, size_t n);
void nmzo_go_seed(nmzo_go_rng *rng, int64_t seed);
int64_t nmzo_go_int63n(nmzo_go_rng *rng, int64_t n);
int64_t nmzo_go_intn(nmzo_go_rng *rng, int64_t n);
int64_t nmzo_replayable_interval(const uint8_t *seed, size_t seed_len, const uint8_t *hint, size_t hint_len,
                                 int64_t max_interval);
void nmzo_replayable_sweep(const uint32_t *seed_off, const uint8_t *seed_bytes, uint64_t n_seeds,
                           const uint32_t *hint_off, const uint8_t *hint_bytes, uint32_t n_events,
                           int64_t max_interval, nmz_sched_stats *stats, int64_t *delays, uint64_t n_dump, int nthreads);
int nmzo_random_params(int64_t min_ns, int64_t max_ns, double p, nmz_random_params *out);
int nmzo_random_decide(uint64_t seed, uint64_t evhash, uint8_t evclass, const nmz_random_params *p, int64_t *delay,
                       int *fault);
void nmzo_random_sweep(uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash, const uint8_t *evclass,
                       uint32_t n_events, const nmz_random_params *p, nmz_sched_stats *stats, int64_t *delays,
                       uint8_t *faults, uint64_t n_dump, int nthreads);
void nmzo_topk_from_stats(const nmz_sched_stats *stats, uint64_t n, uint64_t seed0, uint32_t k, nmz_topk_entry *out);
uint64_t nmzo_levenshtein(const uint64_t *a, uint64_t n, const uint64_t *b, uint64_t m);
uint32_t nmzo_levenshtein_banded(const uint64_t *a, uint64_t n, const uint64_t *b, uint64_t m, uint32_t w);
void nmzo_ed_allpairs_knn(const uint64_t *off, const uint64_t *sym, uint32_t n, uint32_t w, uint32_t k,
                          uint32_t *ids, uint32_t *dist, int nthreads);

int main(void) {
    nmzo_init();
    int bad = 0;
    bad |= nmzo_fnv1a64((const uint8_t *)"a", 1) != 0xaf63dc4c8601ec8cULL;
    nmzo_go_rng r;
    int64_t seeds[] = {0, 1, -1, INT64_MIN, INT64_MAX, 2147483647, -2147483647};
    for (unsigned i = 0; i < sizeof seeds / sizeof seeds[0]; i++) {
        nmzo_go_seed(&r, seeds[i]);
        for (int j = 0; j < 700; j++) {
            int64_t v = nmzo_go_int63n(&r, (1LL << 62) + 1);
            bad |= v < 0 || v > (1LL << 62);
            v = nmzo_go_intn(&r, 999);
            bad |= v < 0 || v >= 999;
        }
    }
    bad |= nmzo_replayable_interval((const uint8_t *)"", 0, (const uint8_t *)"", 0, 0) != 0;
    (void)nmzo_replayable_interval((const uint8_t *)"foobar", 6, (const uint8_t *)"h", 1, -1);
    uint32_t soff[4] = {0, 0, 3, 9}, hoff[3] = {0, 5, 5};
    const uint8_t sb[] = "abcdefghi", hb[] = "hintx";
    nmz_sched_stats st[3];
    int64_t dl[16];
    nmzo_replayable_sweep(soff, sb, 3, hoff, hb, 2, 100000000, st, dl, 3, 2);
    nmzo_replayable_sweep(soff, sb, 3, hoff, hb, 0, 100000000, st, NULL, 0, 1);
    nmz_random_params p;
    bad |= nmzo_random_params(0, (1LL << 62) + 1, 0.5, &p) != 0;
    uint64_t eh[5] = {1, 2, 3, UINT64_MAX, 0};
    uint8_t ec[5] = {0, 1, 2, 3, 2};
    uint8_t fl[10];
    nmzo_random_sweep(UINT64_MAX - 1, 2, eh, ec, 5, &p, st, dl, fl, 2, 2);
    nmzo_random_sweep(0, 2, eh, ec, 0, &p, st, NULL, NULL, 0, 1);
    for (int i = 0; i < 50; i++) {
        int64_t d;
        int f;
        nmzo_random_decide((uint64_t)i, eh[i % 5], ec[i % 5], &p, &d, &f);
    }
    nmz_topk_entry tk[8];
    nmzo_topk_from_stats(st, 2, 7, 8, tk);
    uint64_t a[6] = {1, 2, 3, 4, 5, 6}, b[4] = {1, 3, 4, 9};
    bad |= nmzo_levenshtein(a, 6, b, 4) != 3;
    bad |= nmzo_levenshtein(a, 0, b, 0) != 0;
    for (uint32_t w = 0; w < 10; w++) (void)nmzo_levenshtein_banded(a, 6, b, 4, w);
    (void)nmzo_levenshtein_banded(a, 0, b, 4, 2);
    uint64_t off[5] = {0, 6, 6, 10, 12}, sym[12] = {1, 2, 3, 4, 5, 6, 1, 3, 4, 9, 7, 7};
    uint32_t ids[4 * 6], ds[4 * 6];
    nmzo_ed_allpairs_knn(off, sym, 4, 3, 6, ids, ds, 2);
    nmzo_ed_allpairs_knn(off, sym, 4, 0, 1, ids, ds, 1);
    if (bad) {
        fprintf(stderr, "oracle sanity checks failed\n");
        return 1;
    }
    printf("oracle checks ok\n");
    return 0;
}
