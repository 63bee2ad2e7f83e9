// Asynchronous request batcher (product code, include/l7gpu.h l7g_batcher_*).
//
// Envoy's HTTP filter asks for one verdict per request from a worker's event
// loop (envoy/cilium_l7policy.cc:127-182).  One device launch per request is
// all latency and no throughput, so callers submit requests here instead:
// each is copied into the pending batch, and a flusher thread classifies the
// batch with one l7g_classify_host launch as soon as max_requests are pending
// or the oldest request has waited max_wait_us.  Callbacks run on the
// flusher thread in submission order; the caller resumes its stream from
// there (Envoy: post continueDecoding / sendLocalReply to the worker's
// dispatcher).
#include <chrono>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"

namespace {

struct Batch {
    std::vector<uint8_t> arena;
    std::vector<uint64_t> off;
    std::vector<uint32_t> len, conn;
    std::vector<l7g_done_fn> fn;
    std::vector<void *> ctx;
    void clear() {
        arena.clear();
        off.clear();
        len.clear();
        conn.clear();
        fn.clear();
        ctx.clear();
    }
    size_t n() const { return off.size(); }
};

}  // namespace

struct l7g_batcher {
    l7g_engine *e = nullptr;
    uint32_t max_n = 1;
    std::chrono::microseconds max_wait{0};
    std::mutex mu;
    std::condition_variable cv, done_cv;
    Batch cur;
    std::chrono::steady_clock::time_point first;
    bool stop = false, flush_now = false;
    uint64_t submitted = 0, completed = 0, launches = 0;
    std::thread th;

    void Run() {
        Batch work;
        std::vector<uint8_t> v;
        std::vector<int32_t> r;
        std::vector<uint32_t> c;
        std::unique_lock<std::mutex> lk(mu);
        for (;;) {
            while (!stop && !flush_now && cur.n() < max_n) {
                if (cur.n() == 0) cv.wait(lk);
                else if (cv.wait_until(lk, first + max_wait) == std::cv_status::timeout) break;
            }
            if (cur.n() == 0) {
                flush_now = false;
                if (stop) break;
                done_cv.notify_all();
                continue;
            }
            std::swap(work, cur);
            cur.clear();
            flush_now = false;
            lk.unlock();
            const size_t n = work.n();
            v.assign(n, 0);
            r.assign(n, -1);
            c.assign(n, 0);
            const int rc = l7g_classify_host(e, work.arena.data(), work.arena.size(), work.off.data(), work.len.data(),
                                             work.conn.data(), (uint32_t)n, v.data(), r.data(), c.data());
            for (size_t i = 0; i < n; i++) {
                if (rc != 0) work.fn[i](work.ctx[i], L7G_UNSUPPORTED, -1, 0);
                else work.fn[i](work.ctx[i], v[i], r[i], c[i]);
            }
            lk.lock();
            completed += n;
            launches++;
            done_cv.notify_all();
        }
        done_cv.notify_all();
    }
};

extern "C" {

l7g_batcher *l7g_batcher_create(l7g_engine *e, uint32_t max_requests, uint32_t max_wait_us) {
    if (!e) return nullptr;
    auto *b = new l7g_batcher();
    b->e = e;
    b->max_n = max_requests ? max_requests : 1;
    b->max_wait = std::chrono::microseconds(max_wait_us);
    b->th = std::thread([b] { b->Run(); });
    return b;
}

int l7g_batcher_submit(l7g_batcher *b, const uint8_t *req, uint32_t len, uint32_t conn, l7g_done_fn done, void *ctx) {
    std::lock_guard<std::mutex> g(b->mu);
    if (b->stop) return -1;
    Batch &B = b->cur;
    if (B.n() == 0) b->first = std::chrono::steady_clock::now();
    B.off.push_back(B.arena.size());
    B.arena.insert(B.arena.end(), req, req + len);
    B.len.push_back(len);
    B.conn.push_back(conn);
    B.fn.push_back(done);
    B.ctx.push_back(ctx);
    b->submitted++;
    if (B.n() == 1 || B.n() >= b->max_n) b->cv.notify_one();
    return 0;
}

int l7g_batcher_flush(l7g_batcher *b) {
    std::unique_lock<std::mutex> lk(b->mu);
    const uint64_t target = b->submitted;
    b->flush_now = true;
    b->cv.notify_one();
    b->done_cv.wait(lk, [&] { return b->completed >= target; });
    return 0;
}

void l7g_batcher_destroy(l7g_batcher *b) {
    if (!b) return;
    {
        std::lock_guard<std::mutex> g(b->mu);
        b->stop = true;
        b->flush_now = true;
    }
    b->cv.notify_one();
    b->th.join();
    delete b;
}

void l7g_batcher_stats(l7g_batcher *b, uint64_t *requests, uint64_t *launches) {
    std::lock_guard<std::mutex> g(b->mu);
    if (requests) *requests = b->completed;
    if (launches) *launches = b->launches;
}

}  // extern "C"
