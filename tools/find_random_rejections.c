/* Test-vector search (test infrastructure): event hashes whose Intn(999) fault draw is rejected by
 * Go's Int31n bound under the random policy's per-event seeding, for
 *   type R: a ranged delay (one Int63n draw, accepted) followed by the fault draw, and
 *   type F: a fixed-duration class (no delay draw) followed by the fault draw.
 * Uses the CPU oracle (oracle/nmz_oracle.c): nmzo_random_decide returns the number of Go outputs a
 * decision consumed, so a rejected fault draw shows as 3 (type R) or 2 (type F) outputs.
 * Output: JSON lines {"type":..,"seed":..,"evhash":..,"outputs":..} for tests/golden/random_rejections.json.
 * Build: gcc -O2 -fopenmp tools/find_random_rejections.c -Loracle/build -lnmz_oracle -o /tmp/frr */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include "../include/nmz_gpu.h"

void nmzo_init(void);
int nmzo_random_params(int64_t min_ns, int64_t max_ns, double p, nmz_random_params *out);
int nmzo_random_decide(uint64_t seed, uint64_t evhash, uint8_t evclass, const nmz_random_params *p,
                       int64_t *delay, int *fault);

static uint64_t splitmix(uint64_t x) {
    uint64_t z = x + 0x9E3779B97F4A7C15ULL;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
    return z ^ (z >> 31);
}

int main(int argc, char **argv) {
    const uint64_t seed = argc > 1 ? strtoull(argv[1], 0, 0) : 0x5EED;
    const uint64_t n = argc > 2 ? strtoull(argv[2], 0, 0) : 100000000ULL;
    const int want = argc > 3 ? atoi(argv[3]) : 4;
    nmzo_init();
    nmz_random_params ranged, fixed;
    nmzo_random_params(30000000, 100000000, 0.1, &ranged);
    nmzo_random_params(5000000, 5000000, 0.1, &fixed);
    int found_r = 0, found_f = 0;
#pragma omp parallel for schedule(dynamic, 65536)
    for (uint64_t i = 0; i < n; i++) {
        if (found_r >= want && found_f >= want) continue;
        const uint64_t eh = splitmix(i);
        int64_t d;
        int f;
        const int outs_r = nmzo_random_decide(seed, eh, NMZ_EV_FAULTABLE, &ranged, &d, &f);
        const int outs_f = nmzo_random_decide(seed, eh, NMZ_EV_FAULTABLE, &fixed, &d, &f);
        if (outs_r <= 2 && outs_f <= 1) continue;
#pragma omp critical
        {
            if (outs_r > 2 && found_r < want) {
                found_r++;
                printf("{\"type\": \"ranged\", \"seed\": %llu, \"evhash\": %llu, \"outputs\": %d}\n",
                       (unsigned long long)seed, (unsigned long long)eh, outs_r);
                fflush(stdout);
            }
            if (outs_f > 1 && found_f < want) {
                found_f++;
                printf("{\"type\": \"fixed\", \"seed\": %llu, \"evhash\": %llu, \"outputs\": %d}\n",
                       (unsigned long long)seed, (unsigned long long)eh, outs_f);
                fflush(stdout);
            }
        }
    }
    return 0;
}
