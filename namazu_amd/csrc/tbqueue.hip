// Time-bounded queue: the delivery half of the online decision path (host code only).
//
// The reference's queue (util/queue/impl.go:64-128, BasicTBQueue) has two release rules:
//   * ranged items (min != max, impl.go:120-126): a goroutine per item, `<-time.After(duration); dequeueChan <-
//     item`, so each is released at its own enqueue + duration;
//   * fixed-duration items (min == max, impl.go:77-89,117-119): ONE goroutine over an infinite channel takes the
//     next item, waits `<-time.After(d)` from the moment it took it, hands it over, and only then takes the next.
//     A burst of n fixed items enqueued together is therefore released at d, 2d, ..., nd: item k's timer starts
//     at max(its enqueue, item k-1's release). This is the random policy's default (maxInterval defaults to
//     minInterval, randompolicy.go:171-178).
// Here one timer thread owns a min-heap of (due time, enqueue sequence) for the ranged items and a FIFO lane for
// the fixed ones, whose head's due time is max(head enqueue, previous fixed release) + d with the previous
// release taken as the instant it actually happened (the goroutine's next time.After starts after its send).
// Every item whose due time has come moves to a FIFO that consumers block on (ActionChan). The reference's
// handoff is an unbuffered channel, so a consumer slower than d would stall its fixed lane further; here the
// release is the handoff (the consumer side is a buffered deque), which equals the reference whenever the
// consumer is waiting in its receive. Due times are CLOCK_MONOTONIC nanoseconds
// (std::chrono::steady_clock; Python's time.monotonic_ns), so a caller stamps the enqueue time, decides the
// delay (nmz_*_decide_host) and enqueues at enqueue + delay; the item records when it was released, so the
// delivered-delay error (release - due) is exact whatever the consumer does. Equal due times release in
// enqueue order. The timer sleeps until shortly before the earliest due time and busy-waits the rest (no
// sched_yield: under CFS a yielding thread can lose the CPU for a whole time slice), with a 1 ns timer slack
// (the default 50 us slack makes a timed wait wake late).
#include <sys/prctl.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <queue>
#include <thread>
#include <vector>

#include "nmz_common.h"

namespace nmz {

static inline int64_t mono_ns() {
    return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

struct TbItem {
    int64_t due;
    uint64_t seq, id;
    bool operator>(const TbItem &o) const { return due != o.due ? due > o.due : seq > o.seq; }
};
struct TbFixed {
    int64_t enqueued, duration;
    uint64_t seq, id;
};
struct TbReady {
    uint64_t id;
    int64_t due, released;
};

constexpr int64_t TB_SPIN_NS = 100'000;  // sleep until this much before the due time, then spin

}  // namespace nmz

struct nmz_tbqueue {
    std::mutex mu;
    std::condition_variable timer_cv, ready_cv;
    std::priority_queue<nmz::TbItem, std::vector<nmz::TbItem>, std::greater<nmz::TbItem>> heap;
    std::deque<nmz::TbFixed> fixed;         // the fixed-duration lane (impl.go:77-89), in enqueue order
    int64_t fixed_last_release = INT64_MIN;  // when the lane last handed an item over
    std::deque<nmz::TbReady> ready;
    uint64_t seq = 0, n_enq = 0, n_rel = 0, n_deq = 0;

    // due time of the fixed lane's head: its timer starts when the lane takes it, i.e. at max(enqueue, last release)
    int64_t fixed_due() const {
        const nmz::TbFixed &f = fixed.front();
        return std::max(f.enqueued, fixed_last_release) + f.duration;
    }
    // the next item to release: 0 = none, 1 = the heap's top, 2 = the fixed lane's head (by due time, then seq)
    int next(int64_t *due) const {
        const bool h = !heap.empty(), f = !fixed.empty();
        if (!h && !f) return 0;
        const int64_t fd = f ? fixed_due() : 0;
        if (h && (!f || heap.top().due < fd || (heap.top().due == fd && heap.top().seq < fixed.front().seq))) {
            *due = heap.top().due;
            return 1;
        }
        *due = fd;
        return 2;
    }
    bool stop = false;
    uint32_t users = 0;              // calls inside dequeue (destroy waits for them to leave before deleting)
    std::condition_variable idle_cv;
    std::thread timer;

    void loop() {
        (void)prctl(PR_SET_TIMERSLACK, 1UL, 0UL, 0UL, 0UL);
        std::unique_lock<std::mutex> lk(mu);
        while (!stop) {
            int64_t due = 0;
            if (!next(&due)) {
                timer_cv.wait(lk);
                continue;
            }
            int64_t now = nmz::mono_ns();
            if (due - now > nmz::TB_SPIN_NS) {
                timer_cv.wait_until(lk, std::chrono::steady_clock::time_point(
                                            std::chrono::nanoseconds(due - nmz::TB_SPIN_NS)));
                continue;  // an earlier item may have arrived
            }
            if (now < due) {
                lk.unlock();
                while (nmz::mono_ns() < due) __builtin_ia32_pause();
                lk.lock();
                now = nmz::mono_ns();
            }
            bool any = false;
            for (int which; (which = next(&due)) != 0 && due <= now; any = true, ++n_rel) {
                if (which == 1) {
                    const nmz::TbItem it = heap.top();
                    heap.pop();
                    ready.push_back(nmz::TbReady{it.id, it.due, now});
                } else {  // a zero-duration successor is due at once, so it leaves in this same pass
                    ready.push_back(nmz::TbReady{fixed.front().id, due, now});
                    fixed.pop_front();
                    fixed_last_release = now;
                }
            }
            if (any) ready_cv.notify_all();
        }
    }
};

using namespace nmz;

extern "C" {

int nmz_tbqueue_create(nmz_tbqueue **out) {
    NMZ_CHECK(out != nullptr, "out is NULL");
    auto *q = new nmz_tbqueue();
    q->timer = std::thread([q] { q->loop(); });
    *out = q;
    return NMZ_OK;
}

int nmz_tbqueue_close(nmz_tbqueue *q) {
    NMZ_CHECK(q != nullptr, "queue is NULL");
    {
        std::lock_guard<std::mutex> lk(q->mu);
        q->stop = true;
    }
    q->timer_cv.notify_all();
    q->ready_cv.notify_all();  // blocked consumers return NMZ_EAGAIN ("queue is closed")
    return NMZ_OK;
}

int nmz_tbqueue_destroy(nmz_tbqueue *q) {
    if (!q) return NMZ_OK;
    nmz_tbqueue_close(q);
    q->timer.join();
    {  // consumers woken by the close leave dequeue before the queue (its mutex and condition variables) goes
        std::unique_lock<std::mutex> lk(q->mu);
        q->idle_cv.wait(lk, [q] { return q->users == 0; });
    }
    delete q;
    return NMZ_OK;
}

int64_t nmz_monotonic_ns(void) { return mono_ns(); }

int nmz_tbqueue_enqueue(nmz_tbqueue *q, uint64_t id, int64_t due_ns) {
    NMZ_CHECK(q != nullptr, "queue is NULL");
    {
        std::lock_guard<std::mutex> lk(q->mu);
        NMZ_CHECK(!q->stop, "queue is closed");
        q->heap.push(TbItem{due_ns, q->seq++, id});
        ++q->n_enq;
    }
    q->timer_cv.notify_one();
    return NMZ_OK;
}

int nmz_tbqueue_enqueue_fixed(nmz_tbqueue *q, uint64_t id, int64_t enqueued_ns, int64_t duration_ns) {
    NMZ_CHECK(q != nullptr, "queue is NULL");
    NMZ_CHECK(duration_ns >= 0, "negative duration");
    {
        std::lock_guard<std::mutex> lk(q->mu);
        NMZ_CHECK(!q->stop, "queue is closed");
        q->fixed.push_back(TbFixed{enqueued_ns, duration_ns, q->seq++, id});
        ++q->n_enq;
    }
    q->timer_cv.notify_one();
    return NMZ_OK;
}

int nmz_tbqueue_dequeue(nmz_tbqueue *q, int64_t timeout_ns, uint64_t *id, int64_t *due_ns, int64_t *released_ns) {
    NMZ_CHECK(q && id, "NULL argument");
    std::unique_lock<std::mutex> lk(q->mu);
    ++q->users;
    struct Leave {  // every return path: the last consumer out of a closed queue lets destroy proceed
        nmz_tbqueue *q;
        ~Leave() {
            if (--q->users == 0 && q->stop) q->idle_cv.notify_all();
        }
    } leave{q};
    auto has = [q] { return !q->ready.empty() || q->stop; };
    if (timeout_ns < 0) {
        q->ready_cv.wait(lk, has);
    } else if (!q->ready_cv.wait_for(lk, std::chrono::nanoseconds(timeout_ns), has)) {
        return fail(NMZ_EAGAIN, "nothing released within the timeout");
    }
    if (q->ready.empty()) return fail(NMZ_EAGAIN, "queue is closed");
    const TbReady r = q->ready.front();
    q->ready.pop_front();
    ++q->n_deq;
    *id = r.id;
    if (due_ns) *due_ns = r.due;
    if (released_ns) *released_ns = r.released;
    return NMZ_OK;
}

int nmz_tbqueue_stats(nmz_tbqueue *q, uint64_t *enqueued, uint64_t *released, uint64_t *dequeued) {
    NMZ_CHECK(q != nullptr, "queue is NULL");
    std::lock_guard<std::mutex> lk(q->mu);
    if (enqueued) *enqueued = q->n_enq;
    if (released) *released = q->n_rel;
    if (dequeued) *dequeued = q->n_deq;
    return NMZ_OK;
}

}  // extern "C"
