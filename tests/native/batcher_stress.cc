// Batcher threading on a host-only engine (no GPU needed: every flush is
// answered L7G_UNSUPPORTED, which still runs the lock-free slots, both
// flusher threads, batch-ordered callbacks, flush and backpressure).
// Checks: every request's callback exactly once, a thread's callbacks in its
// submission order, flush() returns only after its requests were answered,
// flush() from a callback returns -1, submit returns -2 while both flushers
// are busy and the open slot is full, and every accepted request is answered.  stdout: one JSON object.
#include <atomic>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"

static std::atomic<uint64_t> g_calls{0};
static std::atomic<int> g_bad{0};
static std::vector<std::atomic<uint32_t>> *g_next;  // per thread: the next sequence number expected
static l7g_batcher *g_b = nullptr;
static std::atomic<int> g_flush_rc{1};

static void done(void *ctx, uint8_t verdict, int32_t rule, uint32_t consumed) {
    const uint64_t v = (uint64_t)(uintptr_t)ctx;
    const uint32_t t = (uint32_t)(v >> 32), seq = (uint32_t)v;
    if (verdict != L7G_UNSUPPORTED || rule != -1 || consumed != 0) g_bad++;
    if ((*g_next)[t].load() != seq) g_bad++;  // out of order or twice
    (*g_next)[t].store(seq + 1);
    if (t == 0 && seq == 7) g_flush_rc = l7g_batcher_flush(g_b);  // re-entry: must not deadlock
    g_calls++;
}

int main() {
    char err[256];
    l7g_engine *e = l7g_engine_create(L7G_HOST_ONLY, err, sizeof err);
    if (!e) { printf("{\"error\": \"%s\"}\n", err); return 1; }
    const int T = 8, N = 20000;
    std::vector<std::atomic<uint32_t>> next(T);
    for (auto &x : next) x = 0;
    g_next = &next;
    g_b = l7g_batcher_create(e, 256, 50);
    std::atomic<int> rejected{0};
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
        th.emplace_back([t, &rejected] {
            uint8_t req[64];
            memset(req, 'a', sizeof req);
            for (uint32_t i = 0; i < (uint32_t)N; i++) {
                int rc;
                while ((rc = l7g_batcher_submit(g_b, req, 16 + (i % 48), 0, done,
                                                (void *)(uintptr_t)((uint64_t)t << 32 | i))) == -2)
                    rejected++, std::this_thread::yield();
                if (rc != 0) { g_bad++; return; }
            }
        });
    for (auto &x : th) x.join();
    const int frc = l7g_batcher_flush(g_b);
    const uint64_t after_flush = g_calls.load();
    uint64_t reqs = 0, launches = 0;
    l7g_batcher_stats(g_b, &reqs, &launches);
    l7g_batcher_destroy(g_b);
    // large requests (1-31 KB): slots fill by bytes before they fill by count,
    // so racing reservations past the arena's end leave holes the flusher
    // closes up -- still every callback once, in each thread's order
    for (auto &x : next) x = 0;
    const uint64_t calls0 = g_calls.load();
    g_b = l7g_batcher_create(e, 64, 50);
    std::vector<std::thread> th2;
    const int N2 = 3000;
    for (int t = 0; t < T; t++)
        th2.emplace_back([t, &rejected] {
            std::vector<uint8_t> req(32768, 'b');
            for (uint32_t i = 0; i < (uint32_t)N2; i++) {
                int rc;
                while ((rc = l7g_batcher_submit(g_b, req.data(), 1000 + (i * 7919u + t * 104729u) % 30000, 0, done,
                                                (void *)(uintptr_t)((uint64_t)t << 32 | i))) == -2)
                    rejected++, std::this_thread::yield();
                if (rc != 0) { g_bad++; return; }
            }
        });
    for (auto &x : th2) x.join();
    l7g_batcher_flush(g_b);
    const uint64_t large_calls = g_calls.load() - calls0;
    l7g_batcher_destroy(g_b);
    // backpressure: callbacks that block until released keep both flushers
    // busy, so the open slot fills (1024 requests for max_requests = 4) and
    // submit refuses; after the release every queued request is answered
    static std::mutex gate;
    static std::atomic<int> slow_calls{0};
    gate.lock();
    l7g_batcher *slow = l7g_batcher_create(e, 4, 50);
    int queued = 0, refused = 0;
    uint8_t one = 'x';
    for (int i = 0; i < 5000; i++) {
        const int rc = l7g_batcher_submit(slow, &one, 1, 0, [](void *, uint8_t, int32_t, uint32_t) {
            std::lock_guard<std::mutex> g(gate);
            slow_calls++;
        }, nullptr);
        if (rc == 0) queued++; else if (rc == -2) refused++;
    }
    gate.unlock();
    l7g_batcher_flush(slow);
    // a request larger than a lane (the slot's bytes / 8) never fits: refused at once
    std::vector<uint8_t> huge(4u << 20, 'h');
    const int huge_rc = l7g_batcher_submit(slow, huge.data(), (uint32_t)huge.size(), 0,
                                           [](void *, uint8_t, int32_t, uint32_t) {}, nullptr);
    const int slow_answered = slow_calls.load();
    const uint32_t slow_max = l7g_batcher_max_requests(slow);
    l7g_batcher_destroy(slow);
    // a batch size past the cap is reduced, and the caller can read what it got
    l7g_batcher *big = l7g_batcher_create(e, 1u << 20, 50);
    const uint32_t big_max = big ? l7g_batcher_max_requests(big) : 0;
    if (big) l7g_batcher_destroy(big);
    l7g_engine_destroy(e);
    printf("{\"calls\": %llu, \"after_flush\": %llu, \"expected\": %d, \"bad\": %d, \"flush_rc\": %d, "
           "\"reentrant_flush_rc\": %d, \"launches\": %llu, \"queued\": %d, \"refused\": %d, \"rejected\": %d, "
           "\"slow_answered\": %d, \"large_calls\": %llu, \"large_expected\": %d, \"huge_rc\": %d, "
           "\"slow_max\": %u, \"big_max\": %u}\n",
           (unsigned long long)g_calls.load(), (unsigned long long)after_flush, T * N, g_bad.load(), frc,
           g_flush_rc.load(), (unsigned long long)launches, queued, refused, rejected.load(), slow_answered,
           (unsigned long long)large_calls, T * N2, huge_rc, slow_max, big_max);
    return 0;
}
