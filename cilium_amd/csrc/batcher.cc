// Asynchronous request batcher (product code, include/l7gpu.h l7g_batcher_*).
//
// Envoy's HTTP filter asks for one verdict per request from a worker's event
// loop (envoy/cilium_l7policy.cc:127-182).  One device launch per request is
// all latency and no throughput, so callers submit requests here instead and
// get a callback.  Layout (round 4):
//   * submit appends to one of kShards pending queues (the calling thread's
//     shard, picked once per thread), each under its own lock, into storage
//     that keeps its capacity between flushes -- eight submitting threads do
//     not serialise on one lock or on a growing vector;
//   * kFlushers flusher threads each take everything pending (once
//     max_requests are pending, the oldest has waited max_wait_us, or a flush
//     is asked for), classify it with one l7g_classify_host call on their own
//     stream and staging, and run its callbacks -- so one batch is on the
//     device while the next is being gathered and launched;
//   * callbacks run on the flusher threads, batch after batch in the order
//     the batches were taken (a thread's requests in submission order); a
//     callback must not call l7g_batcher_flush or l7g_batcher_destroy (both
//     return at once, doing nothing, when called from a flusher thread);
//   * at most max_pending requests wait (max_requests x 64): beyond that
//     submit returns -2 and the caller answers the request itself.
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"

namespace {

constexpr int kShards = 16;
constexpr int kFlushers = 2;
using Clock = std::chrono::steady_clock;

struct Pending {
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len, conn;
    std::vector<l7g_done_fn> fn;
    std::vector<void *> ctx;
    void clear() {  // (capacity kept)
        arena.clear();
        off.clear();
        len.clear();
        conn.clear();
        fn.clear();
        ctx.clear();
    }
    size_t n() const { return off.size(); }
};

struct alignas(64) Shard {
    std::mutex mu;
    Pending q;
};

std::atomic<uint32_t> g_next_shard{0};
thread_local int t_shard = -1;

}  // namespace

struct l7g_batcher {
    l7g_engine *e = nullptr;
    uint32_t max_n = 1;
    uint64_t max_pending = 64;
    std::chrono::microseconds max_wait{0};
    Shard shards[kShards];
    std::atomic<uint64_t> pending{0};
    std::atomic<int64_t> oldest_ns{0};  // steady-clock time of the first pending submission (0: none)
    // flusher coordination
    std::mutex mu;
    std::condition_variable cv, done_cv;
    std::atomic<bool> stop{false};
    uint64_t flush_gen = 0;  // a flush was asked for (flushers take what is pending at once)
    uint64_t submitted = 0, completed = 0, launches = 0;  // (completed / launches under mu)
    std::atomic<uint64_t> n_submitted{0};
    uint64_t take_seq = 0, deliver_seq = 0;  // batch order of callbacks (under mu)
    std::mutex take_mu;                      // one flusher gathers at a time
    std::thread th[kFlushers];

    bool IsFlusher() const {
        for (const auto &t : th)
            if (t.get_id() == std::this_thread::get_id()) return true;
        return false;
    }

    // Moves every shard's pending requests into w (offsets rebased); returns the count.
    size_t Gather(Pending &w) {
        w.clear();
        for (auto &s : shards) {
            std::lock_guard<std::mutex> g(s.mu);
            Pending &q = s.q;
            if (!q.n()) continue;
            const uint64_t base = w.arena.size();
            w.arena.insert(w.arena.end(), q.arena.begin(), q.arena.end());
            for (uint64_t o : q.off) w.off.push_back(base + o);
            w.len.insert(w.len.end(), q.len.begin(), q.len.end());
            w.conn.insert(w.conn.end(), q.conn.begin(), q.conn.end());
            w.fn.insert(w.fn.end(), q.fn.begin(), q.fn.end());
            w.ctx.insert(w.ctx.end(), q.ctx.begin(), q.ctx.end());
            q.clear();
        }
        pending.fetch_sub(w.n());
        oldest_ns.store(pending.load() ? Clock::now().time_since_epoch().count() : 0);
        return w.n();
    }

    void Run() {
        Pending work;
        std::vector<uint8_t> v;
        std::vector<int32_t> r;
        std::vector<uint32_t> c;
        uint64_t seen_flush = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    if (stop && pending.load() == 0) return;
                    const uint64_t p = pending.load();
                    if (p >= max_n || (p && (stop || flush_gen != seen_flush))) break;
                    if (p) {
                        const int64_t o = oldest_ns.load();
                        const auto due = Clock::time_point(Clock::duration(o)) + max_wait;
                        if (o && Clock::now() >= due) break;
                        cv.wait_until(lk, o ? due : Clock::now() + max_wait);
                    } else {
                        if (flush_gen != seen_flush) { seen_flush = flush_gen; done_cv.notify_all(); }
                        cv.wait(lk);
                    }
                }
                seen_flush = flush_gen;
            }
            uint64_t seq;
            {
                std::lock_guard<std::mutex> g(take_mu);
                if (!Gather(work)) continue;
                std::lock_guard<std::mutex> g2(mu);
                seq = take_seq++;
            }
            const size_t n = work.n();
            v.assign(n, 0);
            r.assign(n, -1);
            c.assign(n, 0);
            const int rc = l7g_classify_host(e, work.arena.data(), work.arena.size(), work.off.data(), work.len.data(),
                                             work.conn.data(), (uint32_t)n, v.data(), r.data(), c.data());
            {  // callbacks in batch order
                std::unique_lock<std::mutex> lk(mu);
                done_cv.wait(lk, [&] { return deliver_seq == seq; });
            }
            for (size_t i = 0; i < n; i++) {
                if (rc != 0) work.fn[i](work.ctx[i], L7G_UNSUPPORTED, -1, 0);
                else work.fn[i](work.ctx[i], v[i], r[i], c[i]);
            }
            {
                std::lock_guard<std::mutex> g(mu);
                deliver_seq++;
                completed += n;
                launches++;
            }
            done_cv.notify_all();
            cv.notify_all();  // the other flusher may have work waiting
        }
    }
};

extern "C" {

l7g_batcher *l7g_batcher_create(l7g_engine *e, uint32_t max_requests, uint32_t max_wait_us) {
    if (!e) return nullptr;
    auto *b = new l7g_batcher();
    b->e = e;
    b->max_n = max_requests ? max_requests : 1;
    b->max_pending = (uint64_t)b->max_n * 64;
    b->max_wait = std::chrono::microseconds(max_wait_us);
    for (auto &s : b->shards) {
        s.q.arena.reserve((size_t)b->max_n * 512 / kShards + 4096);
        s.q.off.reserve(b->max_n / kShards + 64);
    }
    for (auto &t : b->th) t = std::thread([b] { b->Run(); });
    return b;
}

int l7g_batcher_submit(l7g_batcher *b, const uint8_t *req, uint32_t len, uint32_t conn, l7g_done_fn done, void *ctx) {
    if (b->stop) return -1;  // (unsynchronised read: a submit racing destroy is the caller's error)
    if (b->pending.load(std::memory_order_relaxed) >= b->max_pending) return -2;
    if (t_shard < 0) t_shard = (int)(g_next_shard.fetch_add(1) % kShards);
    Shard &s = b->shards[t_shard];
    // counted before it is queued, so a gather never takes more than `pending` holds
    b->n_submitted.fetch_add(1);
    const uint64_t p = b->pending.fetch_add(1) + 1;
    {
        std::lock_guard<std::mutex> g(s.mu);
        Pending &q = s.q;
        q.off.push_back(q.arena.size());
        q.arena.insert(q.arena.end(), req, req + len);
        q.len.push_back(len);
        q.conn.push_back(conn);
        q.fn.push_back(done);
        q.ctx.push_back(ctx);
    }
    if (p == 1) {
        int64_t z = 0;
        b->oldest_ns.compare_exchange_strong(z, Clock::now().time_since_epoch().count());
        b->cv.notify_all();
    } else if (p == b->max_n) {
        b->cv.notify_all();
    }
    return 0;
}

int l7g_batcher_flush(l7g_batcher *b) {
    if (b->IsFlusher()) return -1;  // from a callback: it would wait on itself
    std::unique_lock<std::mutex> lk(b->mu);
    const uint64_t target = b->n_submitted.load();
    b->flush_gen++;
    b->cv.notify_all();
    b->done_cv.wait(lk, [&] { return b->completed >= target; });
    return 0;
}

void l7g_batcher_destroy(l7g_batcher *b) {
    if (!b || b->IsFlusher()) return;  // (from a callback: not allowed, see the header)
    {
        std::lock_guard<std::mutex> g(b->mu);
        b->stop = true;
    }
    b->cv.notify_all();
    for (auto &t : b->th) t.join();
    delete b;
}

void l7g_batcher_stats(l7g_batcher *b, uint64_t *requests, uint64_t *launches) {
    std::lock_guard<std::mutex> g(b->mu);
    if (requests) *requests = b->completed;
    if (launches) *launches = b->launches;
}

}  // extern "C"
