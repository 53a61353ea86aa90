// Multi-GPU inside the C ABI: device groups (nmz_open_group / nmz_open_group_rank).
//
// The reference's callers are single Go processes (`nmz run`'s initPolicy, cli/run.go:123-136; `nmz tools
// visualize`, cli/tools/visualize.go:138-172), so the drop-in has to reach every GPU of a node from one
// process. A group holds
//   - one context per device (nmz_open: its own stream and scratch),
//   - one worker thread per device, bound to that device once (cgo migrates the caller's OS thread; the
//     workers do not move, and the devices' host-side work -- plan builds, uploads -- runs in parallel),
//   - one RCCL communicator over the devices, created once (ncclCommInitAll; ncclCommInitRank when each
//     process owns one device, nmz_open_group_rank).
// Work is split into n_shards shards (>= the number of ranks: "virtual" shards, so one GPU runs the sharding
// and merge logic of any shard count); shard s runs on rank s mod n_ranks. The sweeps shard by contiguous
// seed range (dist.py shard_range: sizes differ by <= 1), the all-pairs search by the plan's own query-block
// deal (nmz_ed_allpairs_knn_shard_dev: rotated snake order, nmz_ed_block_shard). Each rank merges its shards' results on its device, one RCCL all_gather
// over xGMI exchanges the ranks' lists (k x 24 B top-k, or N x k x 8 B k-NN keys), and a deterministic merge
// -- (n_fault desc, sum_delay desc, seed asc) / (dist asc, id asc) -- gives every rank the same result.
//
// No rank may leave the others waiting in a collective. Every group call therefore runs its local steps (plan
// builds, shard sweeps, list merges) with their status recorded rather than returned, then enters one small status
// all_gather (group_agree_status) that every rank always enters, and only when every rank succeeded the payload
// collective. The status exchange itself cannot fail before its collective: its device and pinned host buffers are
// allocated when the group opens, and a rank whose staging copy fails leaves the failure sentinel (all ones) that
// its send buffer holds between exchanges, so its peers read a failure. NMZ_GROUP_FAIL (an A/B test knob, read only
// with NMZ_AB=1) injects a local failure at one step -- "sweep", "topk", "ed_search" or "exchange" -- on the rank
// NMZ_GROUP_FAIL_RANK (default 0), and nmz_group_collectives counts the collectives this process entered, so a test
// checks that a failed call keeps the collective sequence in step.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <future>
#include <memory>
#include <thread>
#include <utility>

#include "nmz_common.h"
#include "nmz_internal.h"

namespace nmz {

// One thread bound to one device, running submitted tasks in order.
class DeviceWorker {
  public:
    explicit DeviceWorker(int device) : device_(device), th_([this] { loop(); }) {}
    ~DeviceWorker() {
        {
            std::lock_guard<std::mutex> lk(mu_);
            stop_ = true;
        }
        cv_.notify_one();
        th_.join();
    }
    // the task's status and, on failure, its thread-local error message
    std::future<std::pair<int, std::string>> submit(std::function<int()> f) {
        auto task = std::make_shared<std::packaged_task<std::pair<int, std::string>()>>([f = std::move(f)] {
            const int rc = f();
            return std::make_pair(rc, rc == NMZ_OK ? std::string() : std::string(nmz_last_error()));
        });
        auto fut = task->get_future();
        {
            std::lock_guard<std::mutex> lk(mu_);
            q_.push_back([task] { (*task)(); });
        }
        cv_.notify_one();
        return fut;
    }

  private:
    void loop() {
        (void)hipSetDevice(device_);
        for (;;) {
            std::function<void()> job;
            {
                std::unique_lock<std::mutex> lk(mu_);
                cv_.wait(lk, [this] { return stop_ || !q_.empty(); });
                if (q_.empty()) return;
                job = std::move(q_.front());
                q_.pop_front();
            }
            job();
        }
    }
    int device_;
    std::mutex mu_;
    std::condition_variable cv_;
    std::deque<std::function<void()>> q_;
    bool stop_ = false;
    std::thread th_;  // last: started after the members above exist
};

// words per rank of the status / fingerprint exchange (a status word + nmz_ed_plan_fingerprint's words)
constexpr size_t XW_WORDS = 1 + NMZ_ED_FP_WORDS;

struct GroupMember {
    nmz_ctx *ctx = nullptr;
    int rank = 0;
    ncclComm_t comm = nullptr;
    std::unique_ptr<DeviceWorker> worker;
    DevBuf buf[4];  // group scratch on this device: [0] exchange (send | recv), [1] merge scratch, [2] shard outputs
    // the status exchange, allocated at group open: device send [XW_WORDS] | recv [n_ranks][XW_WORDS], and pinned
    // host staging of the same layout
    DevBuf xw;
    uint64_t *xw_host = nullptr;
};

}  // namespace nmz

struct nmz_group {
    std::vector<nmz::GroupMember> m;  // the devices of this process
    int n_ranks = 1;
    uint32_t n_shards = 1;
    bool multi_process = false;
    std::mutex mu;        // group calls are serialised (their contexts and scratch are the group's own)
    uint32_t n_plans = 0;  // live group plans (nmz_close_group refuses to free a group they still use)
    uint64_t n_coll = 0;   // collectives this process has entered (nmz_group_collectives)
};

namespace nmz {

#define NMZ_NCCL(call)                                                                                   \
    do {                                                                                                 \
        ncclResult_t r_ = (call);                                                                        \
        if (r_ != ncclSuccess) return ::nmz::fail(NMZ_EHIP, std::string(#call) + ": " + ncclGetErrorString(r_)); \
    } while (0)

// run fn(member index) on every member's worker thread, wait for all; the first failure's status and message
// become the caller's (thread-local error)
static int run_all(nmz_group *g, const std::function<int(size_t)> &fn) {
    std::vector<std::future<std::pair<int, std::string>>> fut;
    for (size_t i = 0; i < g->m.size(); ++i) fut.push_back(g->m[i].worker->submit([&fn, i] { return fn(i); }));
    int rc = NMZ_OK;
    std::string msg;
    for (auto &f : fut) {
        auto r = f.get();
        if (r.first != NMZ_OK && rc == NMZ_OK) {
            rc = r.first;
            msg = r.second;
        }
    }
    if (rc != NMZ_OK) return fail(rc, msg);
    return NMZ_OK;
}

// the shards of `rank`: rank, rank + n_ranks, ...
static std::vector<uint32_t> shards_of(const nmz_group *g, int rank) {
    std::vector<uint32_t> s;
    for (uint32_t x = (uint32_t)rank; x < g->n_shards; x += (uint32_t)g->n_ranks) s.push_back(x);
    return s;
}

// [lo, hi) of shard s of `total` units (sizes differ by <= 1; namazu_amd/dist.py shard_range)
static std::pair<uint64_t, uint64_t> shard_range(uint64_t total, uint32_t n, uint32_t s) {
    const uint64_t base = total / n, extra = total % n;
    const uint64_t lo = s * base + std::min<uint64_t>(s, extra);
    return {lo, lo + base + (s < extra ? 1 : 0)};
}

// All-gather `bytes` from every member's send buffer into its recv buffer ([n_ranks][bytes], rank order), on the
// members' streams (ordered after the work that filled send). One RCCL group call covers every local device.
static int group_allgather(nmz_group *g, const std::vector<void *> &send, const std::vector<void *> &recv,
                           size_t bytes) {
    ++g->n_coll;
    NMZ_NCCL(ncclGroupStart());
    for (size_t i = 0; i < g->m.size(); ++i) {
        GroupMember &mb = g->m[i];
        if (hipSetDevice(mb.ctx->device) != hipSuccess) {
            (void)ncclGroupEnd();
            return fail(NMZ_EHIP, "hipSetDevice failed");
        }
        const ncclResult_t r = ncclAllGather(send[i], recv[i], bytes, ncclUint8, mb.comm, mb.ctx->stream);
        if (r != ncclSuccess) {
            (void)ncclGroupEnd();
            return fail(NMZ_EHIP, std::string("ncclAllGather: ") + ncclGetErrorString(r));
        }
    }
    NMZ_NCCL(ncclGroupEnd());
    return NMZ_OK;
}

// NMZ_GROUP_FAIL=<step> (with NMZ_AB=1): member `mb` fails locally at `step` when it is rank NMZ_GROUP_FAIL_RANK
static int injected(const GroupMember &mb, const char *step) {
    const char *e = ab_env("NMZ_GROUP_FAIL");
    if (!e || std::strcmp(e, step) != 0) return NMZ_OK;
    const char *r = ab_env("NMZ_GROUP_FAIL_RANK");
    if ((r ? atoi(r) : 0) != mb.rank) return NMZ_OK;
    return fail(NMZ_EHIP, std::string("injected failure at ") + step + " (NMZ_GROUP_FAIL) on rank " +
                              std::to_string(mb.rank));
}

// Every member's `words` u64 (its local status first) to every member, rank order: one small RCCL all_gather that
// every member always enters (its buffers were allocated at group open), so no rank is left waiting in a collective
// another rank skipped. A member whose staging copy fails still enters: its send buffer holds the failure sentinel
// (all ones, re-armed after every exchange), which its peers read as a failed status. all[i] = [n_ranks][words] as
// member i received it; the first local failure is returned after the collective.
static int group_exchange_words(nmz_group *g, const std::vector<std::vector<uint64_t>> &mine, size_t words,
                                std::vector<std::vector<uint64_t>> &all) {
    const size_t R = (size_t)g->n_ranks, n = g->m.size();
    if (words > XW_WORDS) return fail(NMZ_EINVAL, "status exchange too wide");  // a static property of the callers
    std::vector<void *> send(n), recv(n);
    std::vector<int> lrc(n, NMZ_OK);
    std::vector<std::string> lmsg(n);
    all.assign(n, std::vector<uint64_t>(R * words, UINT64_MAX));
    (void)run_all(g, [&](size_t i) {
        GroupMember &mb = g->m[i];
        send[i] = mb.xw.as<uint64_t>();
        recv[i] = mb.xw.as<uint64_t>() + XW_WORDS;
        std::memcpy(mb.xw_host, mine[i].data(), words * 8);
        int rc = injected(mb, "exchange");
        if (rc == NMZ_OK && hipMemcpyAsync(send[i], mb.xw_host, words * 8, hipMemcpyHostToDevice, mb.ctx->stream) !=
                                hipSuccess)
            rc = fail(NMZ_EHIP, "staging the status exchange failed");
        if (rc != NMZ_OK) {
            lrc[i] = rc;
            lmsg[i] = nmz_last_error();
        }
        return NMZ_OK;
    });
    int rc = group_allgather(g, send, recv, words * 8);
    std::string msg = rc == NMZ_OK ? std::string() : std::string(nmz_last_error());
    if (rc == NMZ_OK) {
        rc = run_all(g, [&](size_t i) {
            GroupMember &mb = g->m[i];
            hipStream_t st = mb.ctx->stream;
            uint64_t *h = mb.xw_host + XW_WORDS;
            NMZ_HIP(hipMemcpyAsync(h, recv[i], R * words * 8, hipMemcpyDeviceToHost, st));
            NMZ_HIP(hipMemsetAsync(send[i], 0xff, XW_WORDS * 8, st));  // re-arm the sentinel for the next exchange
            NMZ_HIP(hipStreamSynchronize(st));
            std::memcpy(all[i].data(), h, R * words * 8);
            return NMZ_OK;
        });
        if (rc != NMZ_OK) msg = nmz_last_error();
    }
    for (size_t i = 0; i < n; ++i)
        if (lrc[i] != NMZ_OK) return fail(lrc[i], lmsg[i]);
    return rc == NMZ_OK ? NMZ_OK : fail(rc, msg);
}

// after a step each member ran locally (status st[i], message msg[i]): every rank learns every rank's status;
// NMZ_OK only when all succeeded, else the first failure (this process's own message when it failed here)
static int group_agree_status(nmz_group *g, const std::vector<int> &st, const std::vector<std::string> &msg,
                              const char *what) {
    std::vector<std::vector<uint64_t>> mine(g->m.size()), all;
    for (size_t i = 0; i < g->m.size(); ++i) mine[i] = {(uint64_t)(int64_t)st[i]};
    const int xrc = group_exchange_words(g, mine, 1, all);
    for (size_t i = 0; i < g->m.size(); ++i)
        if (st[i] != NMZ_OK) return fail(st[i], msg[i]);
    if (xrc != NMZ_OK) return xrc;
    for (size_t r = 0; r < all[0].size(); ++r)
        if (all[0][r] != 0)
            return fail(all[0][r] == UINT64_MAX ? NMZ_EHIP : (int)(int64_t)all[0][r],
                        std::string(what) + " failed on rank " + std::to_string(r));
    return NMZ_OK;
}

// runs fn(member index) on every member and records its status instead of returning it (the call continues to
// the status agreement whatever happened locally)
static void run_all_local(nmz_group *g, std::vector<int> &st, std::vector<std::string> &msg,
                          const std::function<int(size_t)> &fn) {
    st.assign(g->m.size(), NMZ_OK);
    msg.assign(g->m.size(), std::string());
    (void)run_all(g, [&](size_t i) {
        st[i] = fn(i);
        if (st[i] != NMZ_OK) msg[i] = nmz_last_error();
        return NMZ_OK;
    });
}

// the member whose copy of a merged result goes to the host: every rank of a multi-process group returns
// its own (identical) copy; in one process, member 0's
static bool reports(const nmz_group *g, size_t i) { return g->multi_process || i == 0; }

static int group_init_member(nmz_group *g, int device, int rank) {
    GroupMember mb;
    NMZ_TRY(nmz_open(device, &mb.ctx));
    mb.rank = rank;
    mb.worker.reset(new DeviceWorker(device));
    g->m.push_back(std::move(mb));
    // the status exchange's buffers, armed with the failure sentinel
    GroupMember &m = g->m.back();
    const size_t bytes = (1 + (size_t)g->n_ranks) * XW_WORDS * 8;
    NMZ_HIP(hipSetDevice(device));
    NMZ_TRY(m.xw.ensure(bytes));
    NMZ_HIP(hipHostMalloc((void **)&m.xw_host, bytes, hipHostMallocDefault));
    NMZ_HIP(hipMemset(m.xw.ptr, 0xff, XW_WORDS * 8));
    return NMZ_OK;
}

static void group_free(nmz_group *g) {
    for (GroupMember &mb : g->m) {
        if (mb.ctx) {
            (void)hipSetDevice(mb.ctx->device);
            (void)hipDeviceSynchronize();
            for (DevBuf &b : mb.buf) b.release();
            mb.xw.release();
            if (mb.xw_host) (void)hipHostFree(mb.xw_host);
        }
        if (mb.comm) (void)ncclCommDestroy(mb.comm);
        mb.worker.reset();
        if (mb.ctx) (void)nmz_close(mb.ctx);
    }
    delete g;
}

// ---- top-k exchange shared by both sweeps -------------------------------------------------------------
// Member i has written its shards' top-k lists ([n_local][k] at lists_i) unless its sweep failed (st[i]); merge
// them into one list, agree on every rank's status, all_gather the ranks' lists, merge those into the final k and
// copy it to `topk` (host).
static int group_topk_exchange(nmz_group *g, uint32_t k, const std::vector<nmz_topk_entry *> &lists,
                               const std::vector<uint32_t> &n_local, nmz_topk_entry *topk,
                               const std::vector<int> &sweep_st, const std::vector<std::string> &sweep_msg) {
    const size_t R = (size_t)g->n_ranks;
    std::vector<void *> send(g->m.size()), recv(g->m.size());
    std::vector<int> st2;
    std::vector<std::string> msg2;
    run_all_local(g, st2, msg2, [&](size_t i) {
        if (sweep_st[i] != NMZ_OK) return fail(sweep_st[i], sweep_msg[i]);  // the sweep failed here: nothing to merge
        GroupMember &mb = g->m[i];
        NMZ_TRY(injected(mb, "topk"));
        const size_t lb = Carve::bytes_for(k, sizeof(nmz_topk_entry));
        NMZ_TRY(mb.buf[0].ensure(lb + Carve::bytes_for(R * k, sizeof(nmz_topk_entry))));
        NMZ_TRY(mb.buf[1].ensure(Carve::bytes_for(std::max<size_t>(R, n_local[i]) * k + k, sizeof(nmz_topk_entry))));
        Carve cv(mb.buf[0].ptr);
        nmz_topk_entry *s = cv.take<nmz_topk_entry>(k), *r = cv.take<nmz_topk_entry>(R * k);
        send[i] = s;
        recv[i] = r;
        hipStream_t st = mb.ctx->stream;
        if (n_local[i] == 0) {  // no shard on this rank: a list of sentinels
            std::vector<nmz_topk_entry> sent(k);
            for (auto &e : sent) e = nmz_topk_entry{UINT64_MAX, INT64_MIN, 0u, NMZ_NONE};
            NMZ_HIP(hipMemcpyAsync(s, sent.data(), k * sizeof(nmz_topk_entry), hipMemcpyHostToDevice, st));
            NMZ_HIP(hipStreamSynchronize(st));  // pageable source
            return NMZ_OK;
        }
        return topk_merge_lists(st, lists[i], mb.buf[1].as<nmz_topk_entry>(), n_local[i], k, s);
    });
    NMZ_TRY(group_agree_status(g, st2, msg2, "the sweep"));
    NMZ_TRY(group_allgather(g, send, recv, (size_t)k * sizeof(nmz_topk_entry)));
    return run_all(g, [&](size_t i) {
        if (!reports(g, i)) return NMZ_OK;
        GroupMember &mb = g->m[i];
        hipStream_t st = mb.ctx->stream;
        nmz_topk_entry *fin = mb.buf[1].as<nmz_topk_entry>() + R * k;
        // topk_merge_lists overwrites both of its buffers: merge from a copy of the gathered lists
        nmz_topk_entry *a = (nmz_topk_entry *)recv[i];
        NMZ_TRY(topk_merge_lists(st, a, mb.buf[1].as<nmz_topk_entry>(), R, k, fin));
        NMZ_HIP(hipMemcpyAsync(topk, fin, k * sizeof(nmz_topk_entry), hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        return NMZ_OK;
    });
}

}  // namespace nmz

using namespace nmz;

// ---- group plans -------------------------------------------------------------------------------------------
struct nmz_replayable_group_plan {
    nmz_group *g;
    std::vector<nmz_replayable_plan *> p;  // per member
    uint64_t max_seeds_per_shard;
};
struct nmz_random_group_plan {
    nmz_group *g;
    std::vector<nmz_random_plan *> p;
    uint64_t max_seeds_per_shard;
};
struct nmz_ed_group_plan {
    nmz_group *g;
    std::vector<nmz_ed_plan *> p;
    uint32_t n;
    uint32_t opts = 0;  // NMZ_ED_OPT_* of every member's plan
    std::vector<double> upload_ms, gather_ms, build_ms;  // per local member (nmz_ed_group_plan_timing)
};

namespace nmz {

// Per-member shard outputs: stats of the largest local shard and one top-k list per local shard.
struct ShardOut {
    nmz_sched_stats *stats;
    nmz_topk_entry *lists;
};
static int shard_out(GroupMember &mb, uint64_t max_shard, uint32_t n_local, uint32_t k, ShardOut &o) {
    NMZ_TRY(mb.buf[2].ensure(Carve::bytes_for(max_shard + 1, sizeof(nmz_sched_stats)) +
                             Carve::bytes_for((uint64_t)std::max(n_local, 1u) * k + 1, sizeof(nmz_topk_entry))));
    Carve cv(mb.buf[2].ptr);
    o.stats = cv.take<nmz_sched_stats>(max_shard + 1);
    o.lists = cv.take<nmz_topk_entry>((uint64_t)std::max(n_local, 1u) * k + 1);
    return NMZ_OK;
}

// One sweep over the group: for every local shard, sweep(member, plan index, lo, n, d_stats, d_topk_list) on
// the member's stream (and its stats to the host), then the top-k exchange.
static int group_sweep(nmz_group *g, uint64_t n_seeds, uint32_t k, nmz_sched_stats *stats, nmz_topk_entry *topk,
                       const std::function<int(size_t, uint64_t, uint64_t, nmz_sched_stats *, nmz_topk_entry *)> &sweep) {
    NMZ_CHECK(k <= 256, "top-k supports k <= 256");
    NMZ_CHECK(k == 0 || topk, "topk is NULL");
    std::vector<nmz_topk_entry *> lists(g->m.size());
    std::vector<uint32_t> n_local(g->m.size());
    std::vector<int> st;
    std::vector<std::string> msg;
    run_all_local(g, st, msg, [&](size_t i) {
        GroupMember &mb = g->m[i];
        NMZ_TRY(injected(mb, "sweep"));
        const std::vector<uint32_t> mine = shards_of(g, mb.rank);
        n_local[i] = (uint32_t)mine.size();
        uint64_t mx = 0;
        for (uint32_t s : mine) {
            const auto r = shard_range(n_seeds, g->n_shards, s);
            mx = std::max(mx, r.second - r.first);
        }
        ShardOut o;
        NMZ_TRY(shard_out(mb, mx, n_local[i], std::max(k, 1u), o));
        lists[i] = o.lists;
        hipStream_t st = mb.ctx->stream;
        for (size_t j = 0; j < mine.size(); ++j) {
            const auto r = shard_range(n_seeds, g->n_shards, mine[j]);
            const uint64_t n = r.second - r.first;
            NMZ_TRY(sweep(i, r.first, n, o.stats, k ? o.lists + j * k : nullptr));
            if (stats && n) {
                NMZ_HIP(hipMemcpyAsync(stats + r.first, o.stats, n * sizeof(nmz_sched_stats), hipMemcpyDeviceToHost,
                                       st));
                NMZ_HIP(hipStreamSynchronize(st));  // o.stats is reused by the next shard
            }
        }
        return NMZ_OK;
    });
    if (k == 0) {  // no collective: each rank reports its own shards
        for (size_t i = 0; i < st.size(); ++i)
            if (st[i] != NMZ_OK) return fail(st[i], msg[i]);
        return NMZ_OK;
    }
    return group_topk_exchange(g, k, lists, n_local, topk, st, msg);
}

static int group_merge_knn(GroupMember &mb, uint64_t *parts, uint32_t n_parts, uint32_t N, uint32_t k,
                           uint64_t *out, uint64_t *tmp) {
    // nmz_knn_merge_dev merges up to 8 lists: fold the parts 8 (then 7 + the running result) at a time
    if (n_parts <= 8) return nmz_knn_merge_dev(mb.ctx, parts, n_parts, N, k, out, nullptr);
    const uint64_t nk = (uint64_t)N * k;
    NMZ_TRY(nmz_knn_merge_dev(mb.ctx, parts, 8, N, k, tmp, nullptr));
    for (uint32_t p = 8; p < n_parts; p += 7) {
        const uint32_t take = std::min(7u, n_parts - p);
        // [running | next parts] must be consecutive: copy the running result in front of them
        uint64_t *front = parts + (uint64_t)(p - 1) * nk;
        NMZ_HIP(hipMemcpyAsync(front, tmp, nk * 8, hipMemcpyDeviceToDevice, mb.ctx->stream));
        NMZ_TRY(nmz_knn_merge_dev(mb.ctx, front, take + 1, N, k, p + take >= n_parts ? out : tmp, nullptr));
    }
    return NMZ_OK;
}

}  // namespace nmz

extern "C" {

int nmz_open_group(uint32_t dev_mask, uint32_t n_shards, nmz_group **out) {
    DeviceRestore dr;  // the caller keeps its own current device
    NMZ_CHECK(out != nullptr, "out is NULL");
    *out = nullptr;
    int n = 0;
    NMZ_HIP(hipGetDeviceCount(&n));
    std::vector<int> devs;
    for (int d = 0; d < 32; ++d)
        if (dev_mask & (1u << d)) {
            NMZ_CHECK(d < n, "dev_mask names a device that does not exist");
            devs.push_back(d);
        }
    NMZ_CHECK(!devs.empty(), "dev_mask is empty");
    auto *g = new nmz_group();
    g->n_ranks = (int)devs.size();
    g->n_shards = n_shards ? n_shards : (uint32_t)devs.size();
    if (g->n_shards < (uint32_t)devs.size()) {
        delete g;
        return fail(NMZ_EINVAL, "n_shards must be 0 or >= the number of devices");
    }
    for (size_t i = 0; i < devs.size(); ++i) {
        const int rc = group_init_member(g, devs[i], (int)i);
        if (rc != NMZ_OK) {
            const std::string msg = nmz_last_error();
            group_free(g);
            return fail(rc, msg);
        }
    }
    std::vector<ncclComm_t> comms(devs.size());
    const ncclResult_t r = ncclCommInitAll(comms.data(), (int)devs.size(), devs.data());
    if (r != ncclSuccess) {
        group_free(g);
        return fail(NMZ_EHIP, std::string("ncclCommInitAll: ") + ncclGetErrorString(r));
    }
    for (size_t i = 0; i < devs.size(); ++i) g->m[i].comm = comms[i];
    *out = g;
    return NMZ_OK;
}

int nmz_group_unique_id(uint8_t *id) {
    NMZ_CHECK(id != nullptr, "id is NULL");
    ncclUniqueId u;
    NMZ_NCCL(ncclGetUniqueId(&u));
    std::memcpy(id, u.internal, NMZ_GROUP_ID_BYTES);
    return NMZ_OK;
}

int nmz_open_group_rank(const uint8_t *id, int n_ranks, int rank, int device, uint32_t n_shards, nmz_group **out) {
    DeviceRestore dr;  // the caller keeps its own current device
    NMZ_CHECK(out && id, "NULL argument");
    *out = nullptr;
    NMZ_CHECK(n_ranks >= 1 && rank >= 0 && rank < n_ranks, "bad rank");
    auto *g = new nmz_group();
    g->n_ranks = n_ranks;
    g->multi_process = true;
    g->n_shards = n_shards ? n_shards : (uint32_t)n_ranks;
    if (g->n_shards < (uint32_t)n_ranks) {
        delete g;
        return fail(NMZ_EINVAL, "n_shards must be 0 or >= n_ranks");
    }
    int rc = group_init_member(g, device, rank);
    if (rc != NMZ_OK) {
        const std::string msg = nmz_last_error();
        group_free(g);
        return fail(rc, msg);
    }
    ncclUniqueId u;
    std::memcpy(u.internal, id, NMZ_GROUP_ID_BYTES);
    (void)hipSetDevice(device);
    const ncclResult_t r = ncclCommInitRank(&g->m[0].comm, n_ranks, u, rank);
    if (r != ncclSuccess) {
        group_free(g);
        return fail(NMZ_EHIP, std::string("ncclCommInitRank: ") + ncclGetErrorString(r));
    }
    *out = g;
    return NMZ_OK;
}

int nmz_close_group(nmz_group *g) {
    DeviceRestore dr;  // the caller keeps its own current device
    if (!g) return NMZ_OK;
    {  // a call already inside the group finishes first (it holds the mutex); no call may start once close has
       // begun (the caller's contract, include/nmz_gpu.h)
        std::lock_guard<std::mutex> lk(g->mu);
        NMZ_CHECK(g->n_plans == 0, "the group still has live plans: destroy them before closing the group");
    }
    group_free(g);
    return NMZ_OK;
}

int nmz_group_collectives(const nmz_group *g, uint64_t *n) {
    NMZ_CHECK(g && n, "NULL argument");
    *n = g->n_coll;
    return NMZ_OK;
}

int nmz_group_info(const nmz_group *g, int *n_ranks, int *n_local_devices, uint32_t *n_shards) {
    NMZ_CHECK(g != nullptr, "group is NULL");
    if (n_ranks) *n_ranks = g->n_ranks;
    if (n_local_devices) *n_local_devices = (int)g->m.size();
    if (n_shards) *n_shards = g->n_shards;
    return NMZ_OK;
}

// ---- replayable ---------------------------------------------------------------------------------------------
int nmz_replayable_group_plan_create(nmz_group *g, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                     uint32_t n_events, int64_t max_interval_ns, uint64_t max_seeds_per_shard,
                                     nmz_replayable_group_plan **out) {
    DeviceRestore dr;
    NMZ_CHECK(g && out, "NULL argument");
    *out = nullptr;
    std::lock_guard<std::mutex> lk(g->mu);
    auto *gp = new nmz_replayable_group_plan();
    gp->g = g;
    gp->p.assign(g->m.size(), nullptr);
    gp->max_seeds_per_shard = max_seeds_per_shard;
    const int rc = run_all(g, [&](size_t i) {
        return nmz_replayable_plan_create(g->m[i].ctx, hint_off, hint_bytes, n_events, max_interval_ns,
                                          max_seeds_per_shard, &gp->p[i]);
    });
    if (rc != NMZ_OK) {
        const std::string msg = nmz_last_error();
        for (auto *p : gp->p) (void)nmz_replayable_plan_destroy(p);
        delete gp;
        return fail(rc, msg);
    }
    ++g->n_plans;
    *out = gp;
    return NMZ_OK;
}

int nmz_replayable_group_plan_destroy(nmz_replayable_group_plan *gp) {
    DeviceRestore dr;
    if (!gp) return NMZ_OK;
    std::lock_guard<std::mutex> lk(gp->g->mu);
    (void)run_all(gp->g, [&](size_t i) { return nmz_replayable_plan_destroy(gp->p[i]); });
    --gp->g->n_plans;
    delete gp;
    return NMZ_OK;
}

int nmz_replayable_group_sweep(nmz_replayable_group_plan *gp, const uint32_t *seed_off, const uint8_t *seed_bytes,
                               uint64_t n_seeds, uint32_t k, nmz_sched_stats *stats, nmz_topk_entry *topk) {
    DeviceRestore dr;
    NMZ_CHECK(gp != nullptr, "plan is NULL");
    NMZ_CHECK(n_seeds == 0 || seed_off, "seed_off is NULL");
    nmz_group *g = gp->g;
    std::lock_guard<std::mutex> lk(g->mu);
    // per member: the seed CSR of the largest local shard
    std::vector<DevBuf> seeds(g->m.size());
    struct Release {
        nmz_group *g;
        std::vector<DevBuf> &b;
        ~Release() {
            for (size_t i = 0; i < b.size(); ++i) {
                (void)hipSetDevice(g->m[i].ctx->device);
                (void)hipStreamSynchronize(g->m[i].ctx->stream);
                b[i].release();
            }
        }
    } rel{g, seeds};
    return group_sweep(g, n_seeds, k, stats, topk,
                       [&](size_t i, uint64_t lo, uint64_t n, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk) {
                           if (n == 0) {  // an empty shard: its top-k list is all sentinels
                               if (!k) return NMZ_OK;
                               return nmz_replayable_sweep_topk_dev(gp->p[i], nullptr, nullptr, 0, lo, k, d_stats,
                                                                    d_topk, nullptr);
                           }
                           NMZ_CHECK(n <= gp->max_seeds_per_shard, "a shard has more seeds than the plan allows");
                           GroupMember &mb = g->m[i];
                           hipStream_t st = mb.ctx->stream;
                           const uint32_t b0 = seed_off[lo], b1 = seed_off[lo + n];
                           std::vector<uint32_t> off(n + 1);
                           for (uint64_t t = 0; t <= n; ++t) off[t] = seed_off[lo + t] - b0;
                           NMZ_TRY(seeds[i].ensure(Carve::bytes_for(n + 1, 4) + Carve::bytes_for(b1 - b0 + 1, 1)));
                           Carve cv(seeds[i].ptr);
                           uint32_t *d_off = cv.take<uint32_t>(n + 1);
                           uint8_t *d_b = cv.take<uint8_t>(b1 - b0 + 1);
                           NMZ_HIP(hipMemcpyAsync(d_off, off.data(), (n + 1) * 4, hipMemcpyHostToDevice, st));
                           if (b1 > b0)
                               NMZ_HIP(hipMemcpyAsync(d_b, seed_bytes + b0, b1 - b0, hipMemcpyHostToDevice, st));
                           if (k)
                               NMZ_TRY(nmz_replayable_sweep_topk_dev(gp->p[i], d_off, d_b, n, lo, k, d_stats, d_topk,
                                                                     nullptr));
                           else
                               NMZ_TRY(nmz_replayable_sweep_dev(gp->p[i], d_off, d_b, n, d_stats, nullptr));
                           NMZ_HIP(hipStreamSynchronize(st));  // `off` is pageable and the CSR buffer is reused
                           return NMZ_OK;
                       });
}

int nmz_replayable_group_sweep_decimal(nmz_replayable_group_plan *gp, uint64_t seed_lo, uint64_t n_seeds, uint32_t k,
                                       nmz_sched_stats *stats, nmz_topk_entry *topk) {
    DeviceRestore dr;
    NMZ_CHECK(gp != nullptr, "plan is NULL");
    nmz_group *g = gp->g;
    std::lock_guard<std::mutex> lk(g->mu);
    return group_sweep(g, n_seeds, k, stats, topk,
                       [&](size_t i, uint64_t lo, uint64_t n, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk) {
                           NMZ_CHECK(n <= gp->max_seeds_per_shard, "a shard has more seeds than the plan allows");
                           return nmz_replayable_sweep_decimal_topk_dev(gp->p[i], seed_lo + lo, n, k, d_stats, d_topk,
                                                                        nullptr);
                       });
}

int nmz_replayable_sweep_topk_group(nmz_group *g, const uint32_t *seed_off, const uint8_t *seed_bytes,
                                    uint64_t n_seeds, const uint32_t *hint_off, const uint8_t *hint_bytes,
                                    uint32_t n_events, int64_t max_interval_ns, uint32_t k, nmz_sched_stats *stats,
                                    nmz_topk_entry *topk) {
    NMZ_CHECK(g != nullptr, "group is NULL");
    const uint64_t per = std::max<uint64_t>((n_seeds + g->n_shards - 1) / g->n_shards, 1);
    nmz_replayable_group_plan *gp = nullptr;
    NMZ_TRY(nmz_replayable_group_plan_create(g, hint_off, hint_bytes, n_events, max_interval_ns, per, &gp));
    const int rc = nmz_replayable_group_sweep(gp, seed_off, seed_bytes, n_seeds, k, stats, topk);
    const std::string msg = rc == NMZ_OK ? std::string() : std::string(nmz_last_error());
    (void)nmz_replayable_group_plan_destroy(gp);
    return rc == NMZ_OK ? NMZ_OK : fail(rc, msg);
}

// ---- random -------------------------------------------------------------------------------------------------
int nmz_random_group_plan_create(nmz_group *g, const uint64_t *evhash, const uint8_t *evclass, uint32_t n_events,
                                 const nmz_random_params *params, uint64_t max_seeds_per_shard,
                                 nmz_random_group_plan **out) {
    DeviceRestore dr;
    NMZ_CHECK(g && out, "NULL argument");
    *out = nullptr;
    std::lock_guard<std::mutex> lk(g->mu);
    auto *gp = new nmz_random_group_plan();
    gp->g = g;
    gp->p.assign(g->m.size(), nullptr);
    gp->max_seeds_per_shard = max_seeds_per_shard;
    const int rc = run_all(g, [&](size_t i) {
        return nmz_random_plan_create(g->m[i].ctx, evhash, evclass, n_events, params, std::max<uint64_t>(max_seeds_per_shard, 1),
                                      &gp->p[i]);
    });
    if (rc != NMZ_OK) {
        const std::string msg = nmz_last_error();
        for (auto *p : gp->p) (void)nmz_random_plan_destroy(p);
        delete gp;
        return fail(rc, msg);
    }
    ++g->n_plans;
    *out = gp;
    return NMZ_OK;
}

int nmz_random_group_plan_destroy(nmz_random_group_plan *gp) {
    DeviceRestore dr;
    if (!gp) return NMZ_OK;
    std::lock_guard<std::mutex> lk(gp->g->mu);
    (void)run_all(gp->g, [&](size_t i) { return nmz_random_plan_destroy(gp->p[i]); });
    --gp->g->n_plans;
    delete gp;
    return NMZ_OK;
}

int nmz_random_group_sweep(nmz_random_group_plan *gp, uint64_t seed0, uint64_t n_seeds, uint32_t k,
                           nmz_sched_stats *stats, nmz_topk_entry *topk) {
    DeviceRestore dr;
    NMZ_CHECK(gp != nullptr, "plan is NULL");
    nmz_group *g = gp->g;
    std::lock_guard<std::mutex> lk(g->mu);
    return group_sweep(g, n_seeds, k, stats, topk,
                       [&](size_t i, uint64_t lo, uint64_t n, nmz_sched_stats *d_stats, nmz_topk_entry *d_topk) {
                           NMZ_CHECK(n <= gp->max_seeds_per_shard, "a shard has more seeds than the plan allows");
                           GroupMember &mb = g->m[i];
                           NMZ_TRY(nmz_random_sweep_dev(gp->p[i], seed0 + lo, n, d_stats, nullptr));
                           if (!k) return NMZ_OK;
                           return nmz_topk_select_dev(mb.ctx, d_stats, n, seed0 + lo, k, d_topk, nullptr);
                       });
}

int nmz_random_sweep_topk_group(nmz_group *g, uint64_t seed0, uint64_t n_seeds, const uint64_t *evhash,
                                const uint8_t *evclass, uint32_t n_events, const nmz_random_params *params,
                                uint32_t k, nmz_sched_stats *stats, nmz_topk_entry *topk) {
    NMZ_CHECK(g != nullptr, "group is NULL");
    const uint64_t per = std::max<uint64_t>((n_seeds + g->n_shards - 1) / g->n_shards, 1);
    nmz_random_group_plan *gp = nullptr;
    NMZ_TRY(nmz_random_group_plan_create(g, evhash, evclass, n_events, params, per, &gp));
    const int rc = nmz_random_group_sweep(gp, seed0, n_seeds, k, stats, topk);
    const std::string msg = rc == NMZ_OK ? std::string() : std::string(nmz_last_error());
    (void)nmz_random_group_plan_destroy(gp);
    return rc == NMZ_OK ? NMZ_OK : fail(rc, msg);
}

// ---- all-pairs banded edit distance k-NN ---------------------------------------------------------------------
int nmz_ed_group_plan_create(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                             uint32_t band, nmz_ed_group_plan **out) {
    return nmz_ed_group_plan_create_opts(g, off, sym, n_traces, band, 0, out);
}

int nmz_ed_group_plan_create_opts(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                                  uint32_t band, uint32_t opts, nmz_ed_group_plan **out) {
    DeviceRestore dr;
    NMZ_CHECK(g && out, "NULL argument");
    *out = nullptr;
    std::lock_guard<std::mutex> lk(g->mu);
    NMZ_CHECK(n_traces == 0 || (off && sym), "NULL argument");
    auto *gp = new nmz_ed_group_plan();
    gp->g = g;
    gp->n = n_traces;
    gp->opts = opts;
    gp->p.assign(g->m.size(), nullptr);
    gp->upload_ms.assign(g->m.size(), 0.0);
    gp->gather_ms.assign(g->m.size(), 0.0);
    gp->build_ms.assign(g->m.size(), 0.0);
    // The store reaches every device as a 1/R share through the device's own PCIe link (rank r uploads symbols
    // [r S, r S + S), S = ceil(total / R), zero-padded) into its slot of a full-store buffer, one RCCL all_gather
    // over xGMI fills the other slots in place, and each device builds the plan from device memory
    // (nmz_ed_plan_create_dev; the plan reads the buffer during the call only). Before, every device pushed the
    // whole store through its own link (configs[2]: 1.6 GB per device, 42 ms of a 59 ms plan). DESIGN.md section 6.
    const uint64_t total = n_traces ? off[n_traces] : 0;
    const uint64_t R = (uint64_t)g->n_ranks, share = std::max<uint64_t>((total + R - 1) / R, 1);
    std::vector<DevBuf> full(g->m.size());
    std::vector<void *> send(g->m.size()), recv(g->m.size());
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point t) { return std::chrono::duration<double, std::milli>(clk::now() - t).count(); };
    // Each step that a rank runs locally (upload, plan build) is followed by an exchange of every rank's status, so
    // a rank that failed does not leave the others waiting in the next collective (and all of them fail); after the
    // build the ranks exchange their plans' fingerprints (nmz_ed_plan_fingerprint) and fail with NMZ_EINVAL when they
    // differ: ranks whose plans took different kernels or stores would not search the same pairs.
    const size_t n = g->m.size();
    std::vector<int> st(n, NMZ_OK);
    std::vector<std::string> msg(n);
    auto local = [&](size_t i, const std::function<int()> &fn) {
        st[i] = fn();
        if (st[i] != NMZ_OK) msg[i] = nmz_last_error();
        return NMZ_OK;
    };
    int rc = run_all(g, [&](size_t i) {
        return local(i, [&] {
            const auto t0 = clk::now();
            GroupMember &mb = g->m[i];
            hipStream_t stm = mb.ctx->stream;
            NMZ_TRY(full[i].ensure(Carve::bytes_for(share * R, 8)));
            uint64_t *d = full[i].as<uint64_t>();
            const uint64_t lo = std::min<uint64_t>((uint64_t)mb.rank * share, total);
            const uint64_t hi = std::min<uint64_t>(lo + share, total);
            if (hi > lo)
                NMZ_HIP(hipMemcpyAsync(d + (uint64_t)mb.rank * share, sym + lo, (hi - lo) * 8, hipMemcpyHostToDevice,
                                       stm));
            if (hi - lo < share)
                NMZ_HIP(hipMemsetAsync(d + (uint64_t)mb.rank * share + (hi - lo), 0, (share - (hi - lo)) * 8, stm));
            NMZ_HIP(hipStreamSynchronize(stm));  // pageable source
            send[i] = d + (uint64_t)mb.rank * share;
            recv[i] = d;
            gp->upload_ms[i] = ms_since(t0);
            return NMZ_OK;
        });
    });
    if (rc == NMZ_OK) rc = group_agree_status(g, st, msg, "the store upload");
    if (rc == NMZ_OK) {
        const auto t0 = clk::now();
        rc = group_allgather(g, send, recv, share * 8);
        if (rc == NMZ_OK)
            rc = run_all(g, [&](size_t i) {
                return local(i, [&] {
                    NMZ_HIP(hipStreamSynchronize(g->m[i].ctx->stream));
                    gp->gather_ms[i] = ms_since(t0);
                    const auto t1 = clk::now();
                    NMZ_TRY(nmz_ed_plan_create_opts(g->m[i].ctx, off, nullptr, full[i].as<uint64_t>(), n_traces, band,
                                                    gp->opts, &gp->p[i]));
                    gp->build_ms[i] = ms_since(t1);
                    return NMZ_OK;
                });
            });
    }
    // the plans' fingerprints, with each rank's build status in front
    if (rc == NMZ_OK) {
        constexpr size_t W = 1 + NMZ_ED_FP_WORDS;
        std::vector<std::vector<uint64_t>> mine(n, std::vector<uint64_t>(W, 0)), all;
        for (size_t i = 0; i < n; ++i) {
            mine[i][0] = (uint64_t)(int64_t)st[i];
            if (st[i] == NMZ_OK) (void)nmz_ed_plan_fingerprint(gp->p[i], mine[i].data() + 1);
        }
        rc = group_exchange_words(g, mine, W, all);
        for (size_t i = 0; rc == NMZ_OK && i < n; ++i)
            if (st[i] != NMZ_OK) rc = fail(st[i], msg[i]);
        for (size_t r = 0; rc == NMZ_OK && r < (size_t)R; ++r) {
            if (all[0][r * W] != 0)
                rc = fail((int)(int64_t)all[0][r * W], "the plan build failed on rank " + std::to_string(r));
            else if (!std::equal(all[0].begin() + r * W, all[0].begin() + (r + 1) * W, all[0].begin()))
                rc = fail(NMZ_EINVAL, "ranks built different edit-distance plans (fingerprint of rank " +
                                          std::to_string(r) + " differs from rank 0's): kernel, band, store or "
                                          "search options disagree");
        }
    }
    (void)run_all(g, [&](size_t i) {  // the plans hold what they need
        (void)hipStreamSynchronize(g->m[i].ctx->stream);
        full[i].release();
        return NMZ_OK;
    });
    if (rc != NMZ_OK) {
        const std::string m = nmz_last_error();
        for (auto *p : gp->p) (void)nmz_ed_plan_destroy(p);
        delete gp;
        return fail(rc, m);
    }
    ++g->n_plans;
    *out = gp;
    return NMZ_OK;
}

int nmz_ed_group_plan_timing(const nmz_ed_group_plan *gp, double *upload_ms, double *gather_ms, double *build_ms) {
    NMZ_CHECK(gp != nullptr, "plan is NULL");
    for (size_t i = 0; i < gp->p.size(); ++i) {
        if (upload_ms) upload_ms[i] = gp->upload_ms[i];
        if (gather_ms) gather_ms[i] = gp->gather_ms[i];
        if (build_ms) build_ms[i] = gp->build_ms[i];
    }
    return NMZ_OK;
}

int nmz_ed_group_plan_destroy(nmz_ed_group_plan *gp) {
    DeviceRestore dr;
    if (!gp) return NMZ_OK;
    std::lock_guard<std::mutex> lk(gp->g->mu);
    (void)run_all(gp->g, [&](size_t i) { return nmz_ed_plan_destroy(gp->p[i]); });
    --gp->g->n_plans;
    delete gp;
    return NMZ_OK;
}

int nmz_ed_group_allpairs_knn(nmz_ed_group_plan *gp, uint32_t k, uint32_t *knn_id, uint32_t *knn_dist) {
    DeviceRestore dr;
    NMZ_CHECK(gp != nullptr, "plan is NULL");
    NMZ_CHECK(k >= 1 && k <= 64, "k must be in [1, 64]");
    nmz_group *g = gp->g;
    std::lock_guard<std::mutex> lk(g->mu);
    const uint32_t N = gp->n;
    if (N == 0) return NMZ_OK;
    const uint64_t nk = (uint64_t)N * k;
    const size_t R = (size_t)g->n_ranks;
    std::vector<void *> send(g->m.size()), recv(g->m.size());
    std::vector<uint64_t *> tmp(g->m.size());
    // 1. each rank's shards into partial lists, merged into its send list (status recorded, then agreed on)
    std::vector<int> lst;
    std::vector<std::string> lmsg;
    run_all_local(g, lst, lmsg, [&](size_t i) {
        GroupMember &mb = g->m[i];
        NMZ_TRY(injected(mb, "ed_search"));
        const std::vector<uint32_t> mine = shards_of(g, mb.rank);
        const uint64_t nl = std::max<size_t>(mine.size(), 1);
        NMZ_TRY(mb.buf[0].ensure(Carve::bytes_for(nk, 8) * (1 + R)));
        NMZ_TRY(mb.buf[2].ensure(Carve::bytes_for(nk * nl, 8) + Carve::bytes_for(nk, 8) * 2));
        Carve c0(mb.buf[0].ptr);
        send[i] = c0.take<uint64_t>(nk);
        recv[i] = c0.take<uint64_t>(nk * R);
        Carve c2(mb.buf[2].ptr);
        uint64_t *parts = c2.take<uint64_t>(nk * nl);
        tmp[i] = c2.take<uint64_t>(nk);
        hipStream_t st = mb.ctx->stream;
        if (mine.empty()) {  // no shard here: empty lists
            NMZ_HIP(hipMemsetAsync(send[i], 0xff, nk * 8, st));
            return NMZ_OK;
        }
        for (size_t j = 0; j < mine.size(); ++j)
            NMZ_TRY(nmz_ed_allpairs_knn_shard_dev(gp->p[i], k, mine[j], g->n_shards, parts + j * nk, nullptr));
        NMZ_TRY(ed_tp_flag_check(gp->p[i], true, st));  // a search whose sizes contradicted its cache fails here
        return group_merge_knn(mb, parts, (uint32_t)mine.size(), N, k, (uint64_t *)send[i], tmp[i]);
    });
    NMZ_TRY(group_agree_status(g, lst, lmsg, "the edit-distance search"));
    // 2. the ranks' lists to every rank (RCCL over xGMI)
    NMZ_TRY(group_allgather(g, send, recv, nk * 8));
    // 3. merge + complete (band + 1 for the pairs no shard listed) + split into ids and distances
    return run_all(g, [&](size_t i) {
        if (!reports(g, i)) return NMZ_OK;
        GroupMember &mb = g->m[i];
        hipStream_t st = mb.ctx->stream;
        uint64_t *fin = (uint64_t *)send[i];  // the send list is no longer needed
        NMZ_TRY(group_merge_knn(mb, (uint64_t *)recv[i], (uint32_t)R, N, k, fin, tmp[i]));
        NMZ_TRY(nmz_ed_knn_fill_dev(gp->p[i], k, fin, nullptr));
        std::vector<uint64_t> h(nk);
        NMZ_HIP(hipMemcpyAsync(h.data(), fin, nk * 8, hipMemcpyDeviceToHost, st));
        NMZ_HIP(hipStreamSynchronize(st));
        for (uint64_t t = 0; t < nk; ++t) {
            const bool none = h[t] == UINT64_MAX;
            if (knn_id) knn_id[t] = none ? NMZ_NONE : (uint32_t)h[t];
            if (knn_dist) knn_dist[t] = none ? NMZ_NONE : (uint32_t)(h[t] >> 32);
        }
        return NMZ_OK;
    });
}

int nmz_ed_allpairs_knn_group(nmz_group *g, const uint64_t *off, const uint64_t *sym, uint32_t n_traces,
                              uint32_t band, uint32_t k, uint32_t *knn_id, uint32_t *knn_dist) {
    NMZ_CHECK(g != nullptr, "group is NULL");
    nmz_ed_group_plan *gp = nullptr;
    NMZ_TRY(nmz_ed_group_plan_create(g, off, sym, n_traces, band, &gp));
    const int rc = nmz_ed_group_allpairs_knn(gp, k, knn_id, knn_dist);
    const std::string msg = rc == NMZ_OK ? std::string() : std::string(nmz_last_error());
    (void)nmz_ed_group_plan_destroy(gp);
    return rc == NMZ_OK ? NMZ_OK : fail(rc, msg);
}

}  // extern "C"
