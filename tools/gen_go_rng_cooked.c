/*
 * Regenerates Go's math/rand `rngCooked` seeding table (Go 1.10,
 * src/math/rand/rng.go) from its documented construction
 * (src/math/rand/gen_cooked.go): seed the additive lagged-Fibonacci
 * generator x_n = x_{n-607} + x_{n-273} (mod 2^64) with srand(1), advance it
 * 7.8e12 steps, and take the resulting 607-word state vector.
 *
 * 7.8e12 sequential steps are replaced by a polynomial jump-ahead:
 *   x^N mod P(x),  P(x) = x^607 - x^334 - 1  over Z/2^64
 * (P is monic, so reduction is exact over the ring).
 *
 * The Go stdlib is not vendored in /root/reference and no Go toolchain is
 * present; several plausible variants of gen_cooked's seeding (shift
 * amounts, masking) are generated and the one that reproduces the
 * published Go KATs (rand.New(rand.NewSource(1)).Int63() =
 * 5577006791947779410, 8674665223082153551, ...) is selected by
 * tools/gen_go_rng_cooked.py.
 *
 * usage: gen_go_rng_cooked <shiftA> <shiftB> <mask_each_step 0|1>
 * prints 607 signed int64 values, one per line. The variant that reproduces
 * the KATs is (20, 10, 0): gen_cooked seeds with 20/10-bit shifts (rng.go's
 * Seed uses 40/20) and the additive recurrence is not masked.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define LEN 607
#define TAP 273
#define M31 2147483647
#define MASK63 0x7fffffffffffffffULL

static int32_t seedrand(int32_t x) {
    const int32_t A = 48271, Q = 44488, R = 3399;
    int32_t hi = x / Q, lo = x % Q;
    x = A * lo - R * hi;
    if (x < 0) x += M31;
    return x;
}

/* r = a*b mod P, all degree < LEN */
static void polymulmod(const uint64_t *a, const uint64_t *b, uint64_t *r) {
    static uint64_t t[2 * LEN];
    memset(t, 0, sizeof t);
    for (int i = 0; i < LEN; i++) {
        if (!a[i]) continue;
        uint64_t ai = a[i];
        for (int j = 0; j < LEN; j++) t[i + j] += ai * b[j];
    }
    /* x^607 = x^334 + 1 : fold from the top down */
    for (int k = 2 * LEN - 2; k >= LEN; k--) {
        uint64_t c = t[k];
        if (!c) continue;
        t[k] = 0;
        t[k - LEN + 334] += c;
        t[k - LEN] += c;
    }
    memcpy(r, t, LEN * sizeof(uint64_t));
}

int main(int argc, char **argv) {
    if (argc != 4) { fprintf(stderr, "usage\n"); return 2; }
    int sa = atoi(argv[1]), sb = atoi(argv[2]), mask_each = atoi(argv[3]);
    uint64_t vec0[LEN];
    int32_t x = 1; /* srand(1): 1 % m = 1, non-zero */
    for (int i = -20; i < LEN; i++) {
        x = seedrand(x);
        if (i >= 0) {
            uint64_t u = (uint64_t)(int64_t)x << sa;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x << sb;
            x = seedrand(x);
            u ^= (uint64_t)(int64_t)x;
            vec0[i] = u;
        }
    }
    /* z_k = y_{k-607}; y_s sits at position (333 - s) mod 607 */
    static uint64_t z[2 * LEN];
    for (int k = 0; k < LEN; k++) {
        int s = k - LEN;
        int p = ((333 - s) % LEN + LEN) % LEN;
        z[k] = vec0[p];
    }
    for (int k = LEN; k < 2 * LEN - 1; k++) {
        uint64_t v = z[k - LEN] + z[k - TAP];
        if (mask_each) v &= MASK63;
        z[k] = v;
    }
    if (mask_each) {
        /* masking each step is not linear over Z/2^64 but is linear over
           Z/2^63: the low 63 bits evolve independently, so reduce mod 2^63 */
    }
    /* r = x^N mod P, N = 7.8e12 */
    const uint64_t N = 7800000000000ULL;
    uint64_t r[LEN], base[LEN], tmp[LEN];
    memset(r, 0, sizeof r); r[0] = 1;
    memset(base, 0, sizeof base); base[1] = 1;
    for (uint64_t e = N; e; e >>= 1) {
        if (e & 1) { polymulmod(r, base, tmp); memcpy(r, tmp, sizeof r); }
        if (e >> 1) { polymulmod(base, base, tmp); memcpy(base, tmp, sizeof base); }
    }
    /* y_t for t = N-607+j  ==  z_{N+j} = sum_i r_i z_{i+j} */
    uint64_t out[LEN];
    for (int j = 0; j < LEN; j++) {
        uint64_t acc = 0;
        for (int i = 0; i < LEN; i++) acc += r[i] * z[i + j];
        if (mask_each) acc &= MASK63;
        /* t = N - 607 + j ; position (333 - t) mod 607 */
        uint64_t t = N - LEN + (uint64_t)j;
        int64_t p = (int64_t)((333 + (uint64_t)LEN * 20000000000ULL - t) % LEN);
        out[p] = acc;
    }
    for (int p = 0; p < LEN; p++) printf("%lld\n", (long long)(int64_t)out[p]);
    return 0;
}
