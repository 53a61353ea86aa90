// Host-only exercise of libnmz_gpu's C ABI under ASan/UBSan (build/host_abi_asan) and TSan (build/host_abi_tsan),
// on a machine without a GPU: argument validation of every entry point, parameter resolution
// (randompolicy.go:223-225,337-339, util/queue/impl.go:36-38), the thread-local error message, and context
// opening failing cleanly when no device is present. Exit status 0 = every check held.
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/nmz_gpu.h"

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                                   \
    do {                                                                           \
        if (!(c)) {                                                                \
            std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            g_fail++;                                                              \
        }                                                                          \
    } while (0)

static void params_cases() {
    nmz_random_params p;
    CHECK(nmz_random_params_resolve(30000000, 100000000, 0.1, &p) == NMZ_OK);
    CHECK(p.min_ns[1] == 24000000 && p.max_ns[1] == 80000000 && p.fault_threshold == 100);
    CHECK(nmz_random_params_resolve(5, 5, 1.0, &p) == NMZ_OK && p.fault_threshold == 1000);
    CHECK(nmz_random_params_resolve(1, 3, 0.999, &p) == NMZ_OK && p.fault_threshold == 999);
    CHECK(nmz_random_params_resolve(-7, 7, 0.0, &p) == NMZ_OK && p.min_ns[1] == -5 && p.max_ns[1] == 5);
    CHECK(nmz_random_params_resolve(INT64_MIN, INT64_MAX, 0.5, &p) == NMZ_OK);
    CHECK(nmz_random_params_resolve(10, 5, 0.1, &p) == NMZ_EINVAL);
    CHECK(std::strstr(nmz_last_error(), "minDuration") != nullptr);
    CHECK(nmz_random_params_resolve(0, 1, -0.01, &p) == NMZ_EINVAL);
    CHECK(nmz_random_params_resolve(0, 1, 1.01, &p) == NMZ_EINVAL);
    CHECK(nmz_random_params_resolve(0, 1, std::nan(""), &p) == NMZ_EINVAL);
    CHECK(std::strstr(nmz_last_error(), "faultActionProbability") != nullptr);
    CHECK(nmz_random_params_resolve(0, 1, 0.5, nullptr) == NMZ_EINVAL);
}

static void null_ctx_cases() {
    uint32_t off[2] = {0, 1};
    uint8_t b[1] = {'x'};
    uint64_t o64[2] = {0, 1}, s64[1] = {7}, keys[8], sig[2];
    uint32_t u32[8];
    int64_t d64[4];
    uint8_t f8[4];
    nmz_sched_stats st[2];
    nmz_topk_entry tk[2];
    nmz_random_params rp;
    nmz_random_params_resolve(1, 2, 0.5, &rp);
    CHECK(nmz_replayable_sweep(nullptr, off, b, 1, off, b, 1, 10, st, nullptr, 0, 0, nullptr) == NMZ_EINVAL);
    CHECK(nmz_replayable_plan_create(nullptr, off, b, 1, 10, 1, nullptr) == NMZ_EINVAL);
    CHECK(nmz_replayable_sweep_dev(nullptr, off, b, 1, st, nullptr) == NMZ_EINVAL);
    CHECK(nmz_replayable_sweep_topk_dev(nullptr, off, b, 1, 0, 1, st, tk, nullptr) == NMZ_EINVAL);
    CHECK(nmz_replayable_decide(nullptr, b, 1, off, b, 1, 10, d64) == NMZ_EINVAL);
    CHECK(nmz_random_sweep(nullptr, 0, 1, s64, f8, 1, &rp, st, nullptr, nullptr, 0, 0, nullptr) == NMZ_EINVAL);
    CHECK(nmz_random_plan_create(nullptr, s64, f8, 1, &rp, 1, nullptr) == NMZ_EINVAL);
    CHECK(nmz_random_sweep_dev(nullptr, 0, 1, st, nullptr) == NMZ_EINVAL);
    CHECK(nmz_random_decide(nullptr, 1, s64, f8, 1, &rp, d64, f8) == NMZ_EINVAL);
    CHECK(nmz_topk_select_dev(nullptr, st, 1, 0, 1, tk, nullptr) == NMZ_EINVAL);
    CHECK(nmz_ed_pairs(nullptr, o64, s64, 1, u32, 1, 0, u32) == NMZ_EINVAL);
    CHECK(nmz_ed_allpairs_knn(nullptr, o64, s64, 1, 8, 1, u32, u32) == NMZ_EINVAL);
    CHECK(nmz_ed_plan_create(nullptr, o64, s64, 1, 8, nullptr) == NMZ_EINVAL);
    CHECK(nmz_ed_allpairs_knn_dev(nullptr, 1, keys, nullptr) == NMZ_EINVAL);
    CHECK(nmz_ed_allpairs_knn_shard_dev(nullptr, 1, 0, 1, keys, nullptr) == NMZ_EINVAL);
    CHECK(nmz_knn_merge_dev(nullptr, keys, 1, 1, 1, keys, nullptr) == NMZ_EINVAL);
    CHECK(nmz_ed_plan_counters(nullptr, keys, nullptr) == NMZ_EINVAL);
    CHECK(nmz_trace_signatures(nullptr, o64, s64, nullptr, 1, sig) == NMZ_EINVAL);
    CHECK(nmz_unique_traces(nullptr, o64, s64, nullptr, 1, u32) == NMZ_EINVAL);
    CHECK(nmz_unique_traces_dev(nullptr, o64, s64, nullptr, 1, 0, sig, u32, nullptr) == NMZ_EINVAL);
    CHECK(nmz_timing_enable(nullptr, 1) == NMZ_EINVAL);
    double ms;
    uint64_t cnt;
    CHECK(nmz_timing_read(nullptr, "x", &ms, &cnt, 0) == NMZ_EINVAL);
    CHECK(nmz_ed_plan_is_fast(nullptr) == 0);
    CHECK(nmz_close(nullptr) == NMZ_OK);
    CHECK(nmz_replayable_plan_destroy(nullptr) == NMZ_OK);
    CHECK(nmz_random_plan_destroy(nullptr) == NMZ_OK);
    CHECK(nmz_ed_plan_destroy(nullptr) == NMZ_OK);
    CHECK(std::strlen(nmz_last_error()) > 0);
}

static void no_device_cases() {
    nmz_ctx *c = reinterpret_cast<nmz_ctx *>(0x1);
    int rc = nmz_open(0, &c);
    // no GPU in this container: a clean error and a NULL context (on a GPU box this opens device 0)
    if (rc == NMZ_OK) {
        CHECK(c != nullptr);
        nmz_close(c);
    } else {
        CHECK(c == nullptr && std::strlen(nmz_last_error()) > 0);
    }
    CHECK(nmz_open(-1, &c) != NMZ_OK && c == nullptr);
    CHECK(nmz_open(0, nullptr) == NMZ_EINVAL);
    int n = -1;
    rc = nmz_device_count(&n);
    CHECK(rc != NMZ_OK || n >= 0);
    CHECK(nmz_device_count(nullptr) == NMZ_EINVAL);
    CHECK(nmz_abi_version() == NMZ_ABI_VERSION);
}

// every thread's nmz_last_error() reports its own latest failure (thread-local), under concurrency
static void thread_local_errors(int n_threads, int iters) {
    std::vector<std::thread> ts;
    for (int t = 0; t < n_threads; ++t) {
        ts.emplace_back([t, iters] {
            nmz_random_params p;
            for (int i = 0; i < iters; ++i) {
                const bool bad_p = ((i + t) % 3) == 0, bad_range = ((i + t) % 3) == 1;
                const int rc = nmz_random_params_resolve(bad_range ? 100 + t : t, 50 + i % 7, bad_p ? 2.0 : 0.25, &p);
                if (bad_p) {
                    CHECK(rc == NMZ_EINVAL && std::strstr(nmz_last_error(), "faultActionProbability"));
                } else if (bad_range) {
                    CHECK(rc == NMZ_EINVAL && std::strstr(nmz_last_error(), "minDuration"));
                } else {
                    CHECK(rc == NMZ_OK && p.fault_threshold == 250);
                }
                CHECK(nmz_ed_pairs(nullptr, nullptr, nullptr, 0, nullptr, 0, 0, nullptr) == NMZ_EINVAL);
                CHECK(std::strstr(nmz_last_error(), "ctx is NULL"));
            }
        });
    }
    for (auto &th : ts) th.join();
}

int main() {
    params_cases();
    null_ctx_cases();
    no_device_cases();
    thread_local_errors(8, 2000);
    if (g_fail) {
        std::fprintf(stderr, "%d checks failed\n", g_fail.load());
        return 1;
    }
    std::printf("host ABI checks ok\n");
    return 0;
}
