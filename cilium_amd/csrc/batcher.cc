// Asynchronous request batcher (product code, include/l7gpu.h l7g_batcher_*).
//
// Envoy's HTTP filter asks for one verdict per request from a worker's event
// loop (envoy/cilium_l7policy.cc:127-182).  One device launch per request is
// all latency and no throughput, so callers submit requests here instead and
// get a callback.  Layout (round 4):
//   * submitters write straight into a pinned batch slot, in the layout the
//     device copy reads (offsets, lengths, connections, request bytes): a
//     compare-and-swap reserves an index and an arena range, the submitting
//     threads copy their bytes in parallel, and no lock is taken;
//   * kFlushers flusher threads each seal the open slot (once max_requests
//     are in it, its first request has waited max_wait_us, or a flush is asked
//     for), open a free one in its place, wait for the sealed slot's last
//     writers, and classify it where it lies -- one copy to the device (none
//     for a small batch), one launch, no gather on the host -- on the
//     flusher's own stream, then run its callbacks; so one batch is on the
//     device while the next fills;
//   * callbacks run on the flusher threads, batch after batch in the order
//     the batches were sealed (a thread's requests in submission order); a
//     callback must not call l7g_batcher_flush or l7g_batcher_destroy (both
//     return at once, doing nothing, when called from a flusher thread);
//   * a slot holds 2 x max_requests requests (at least 1024) and 2 KiB of
//     request bytes per request; when both flushers are busy and the open
//     slot is full, submit returns -2 (backpressure) and the caller answers
//     the request itself.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"
#include "capi_internal.h"

namespace {

constexpr int kFlushers = 2;
constexpr int kSlots = kFlushers + 2;  // one per flusher, the open one, and one ready to open
constexpr uint64_t kBytesMask = (1ull << 40) - 1;  // Slot::resv = count << 40 | arena bytes
constexpr uint32_t kMinSlotRequests = 1024;
constexpr uint64_t kSlotBytesPerRequest = 2048;
using Clock = std::chrono::steady_clock;
enum : int { FREE = 0, OPEN = 1, SEALED = 2 };

int64_t now_ns() { return Clock::now().time_since_epoch().count(); }

struct Slot {
    uint8_t *mem = nullptr;  // pinned; plain malloc when there is no device (a host-only engine)
    bool pinned = false;
    uint64_t *off = nullptr;
    uint32_t *len = nullptr, *conn = nullptr;
    uint8_t *arena = nullptr;
    std::vector<l7g_done_fn> fn;
    std::vector<void *> ctx;
    uint32_t cap_n = 0;
    uint64_t cap_bytes = 0;
    std::atomic<uint64_t> resv{0};
    std::atomic<int32_t> writers{0};  // submitters between their check of `state` and their last store
    std::atomic<int> state{FREE};
    std::atomic<int64_t> first_ns{0};  // when its first request was reserved
};

}  // namespace

struct l7g_batcher {
    l7g_engine *e = nullptr;
    uint32_t max_n = 1;
    std::chrono::microseconds max_wait{0};
    Slot slots[kSlots];
    std::atomic<int> open_idx{0};
    std::atomic<bool> stop{false};
    std::atomic<uint64_t> n_submitted{0};
    // flusher coordination
    std::mutex mu;
    std::condition_variable cv, done_cv;
    uint64_t flush_gen = 0;                  // a flush was asked for: seal what is open at once
    uint64_t completed = 0, launches = 0;    // (under mu)
    uint64_t seal_seq = 0, deliver_seq = 0;  // batch order of callbacks (under mu)
    std::mutex seal_mu;
    std::thread th[kFlushers];

    bool IsFlusher() const {
        for (const auto &t : th)
            if (t.get_id() == std::this_thread::get_id()) return true;
        return false;
    }
    void Wake() {
        // (taken and released so that a flusher between its check and its wait
        // cannot miss the notification)
        { std::lock_guard<std::mutex> g(mu); }
        cv.notify_all();
    }
    uint32_t OpenCount() const { return (uint32_t)(slots[open_idx.load()].resv.load() >> 40); }

    // Seals the open slot if it holds requests and a free slot can take its
    // place; returns its index (and its batch number), or -1.
    int Seal(uint64_t *seq) {
        std::lock_guard<std::mutex> g(seal_mu);
        const int i = open_idx.load();
        Slot &s = slots[i];
        if ((s.resv.load() >> 40) == 0) return -1;
        int j = -1;
        for (int k = 1; k < kSlots && j < 0; k++)
            if (slots[(i + k) % kSlots].state.load() == FREE) j = (i + k) % kSlots;
        if (j < 0) return -1;  // (cannot happen with kSlots = kFlushers + 2; the open slot keeps filling)
        Slot &t = slots[j];
        t.resv.store(0);
        t.first_ns.store(0);
        t.state.store(OPEN);
        open_idx.store(j);
        // seq_cst with the submitters' writers++ then state load: a submitter
        // either sees SEALED and moves on, or is counted in s.writers
        s.state.store(SEALED);
        std::lock_guard<std::mutex> g2(mu);
        *seq = seal_seq++;
        return i;
    }

    void Run() {
        std::vector<uint8_t> v;
        std::vector<int32_t> r;
        std::vector<uint32_t> c;
        {  // this thread's stream and staging, made now rather than under its first batch
            uint8_t vv;
            int32_t rr;
            uint32_t cc;
            const Slot &s0 = slots[0];
            l7g_host_run_pinned(e, 0, 0, s0.off, s0.len, s0.conn, s0.arena, &vv, &rr, &cc);
        }
        uint64_t seen_flush = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    const uint32_t p = OpenCount();
                    if (stop && p == 0) return;
                    if (p >= max_n || (p && (stop || flush_gen != seen_flush))) break;
                    if (p) {
                        int64_t o = slots[open_idx.load()].first_ns.load();
                        if (o == 0) o = now_ns();  // (its first writer has not stamped it yet)
                        const auto due = Clock::time_point(Clock::duration(o)) + max_wait;
                        if (Clock::now() >= due) break;
                        cv.wait_until(lk, due);
                    } else {
                        if (flush_gen != seen_flush) {
                            seen_flush = flush_gen;
                            done_cv.notify_all();
                        }
                        cv.wait_for(lk, std::chrono::milliseconds(100));
                    }
                }
                seen_flush = flush_gen;
            }
            uint64_t seq = 0;
            const int i = Seal(&seq);
            if (i < 0) {  // the other flusher sealed it first
                std::this_thread::yield();
                continue;
            }
            Slot &s = slots[i];
            while (s.writers.load() != 0) std::this_thread::yield();
            const uint64_t rv = s.resv.load();
            const uint32_t n = (uint32_t)(rv >> 40);
            const uint64_t bytes = rv & kBytesMask;
            v.resize(n);
            r.resize(n);
            c.resize(n);
            const int rc = l7g_host_run_pinned(e, n, bytes, s.off, s.len, s.conn, s.arena, v.data(), r.data(), c.data());
            {  // callbacks in batch order
                std::unique_lock<std::mutex> lk(mu);
                done_cv.wait(lk, [&] { return deliver_seq == seq; });
            }
            for (uint32_t k = 0; k < n; k++) {
                if (rc != 0) s.fn[k](s.ctx[k], L7G_UNSUPPORTED, -1, 0);
                else s.fn[k](s.ctx[k], v[k], r[k], c[k]);
            }
            s.state.store(FREE);
            {
                std::lock_guard<std::mutex> g(mu);
                deliver_seq++;
                completed += n;
                launches++;
            }
            done_cv.notify_all();
            cv.notify_all();
        }
    }
};

static void FreeSlots(l7g_batcher *b) {
    for (auto &s : b->slots) {
        if (!s.mem) continue;
        if (s.pinned) l7g_pinned_free(s.mem);
        else free(s.mem);
        s.mem = nullptr;
    }
}

extern "C" {

l7g_batcher *l7g_batcher_create(l7g_engine *e, uint32_t max_requests, uint32_t max_wait_us) {
    if (!e) return nullptr;
    auto *b = new l7g_batcher();
    b->e = e;
    b->max_n = std::min<uint32_t>(max_requests ? max_requests : 1, 1u << 20);
    b->max_wait = std::chrono::microseconds(max_wait_us);
    const uint32_t cap_n = std::max<uint32_t>(2 * b->max_n, kMinSlotRequests);
    const uint64_t cap_bytes = (uint64_t)cap_n * kSlotBytesPerRequest;
    const size_t meta = ((size_t)cap_n * 16 + 255) & ~(size_t)255;
    const size_t total = meta + cap_bytes + 64;  // (+64: aligned 16-byte reads past the last request stay inside)
    for (auto &s : b->slots) {
        s.mem = (uint8_t *)l7g_pinned_alloc(total);
        s.pinned = s.mem != nullptr;
        if (!s.mem) s.mem = (uint8_t *)malloc(total);
        if (!s.mem) {
            FreeSlots(b);
            delete b;
            return nullptr;
        }
        s.off = (uint64_t *)s.mem;
        s.len = (uint32_t *)(s.mem + (size_t)cap_n * 8);
        s.conn = (uint32_t *)(s.mem + (size_t)cap_n * 12);
        s.arena = s.mem + meta;
        s.fn.resize(cap_n);
        s.ctx.resize(cap_n);
        s.cap_n = cap_n;
        s.cap_bytes = cap_bytes;
    }
    b->slots[0].state.store(OPEN);
    for (auto &t : b->th) t = std::thread([b] { b->Run(); });
    return b;
}

int l7g_batcher_submit(l7g_batcher *b, const uint8_t *req, uint32_t len, uint32_t conn, l7g_done_fn done, void *ctx) {
    if (b->stop.load(std::memory_order_relaxed)) return -1;  // (a submit racing destroy is the caller's error)
    if (len > b->slots[0].cap_bytes) return -2;               // never fits a slot
    for (int tries = 0;;) {
        const int i = b->open_idx.load();
        Slot &s = b->slots[i];
        s.writers.fetch_add(1);
        if (s.state.load() != OPEN || b->open_idx.load() != i) {  // sealed under us: take the next one
            s.writers.fetch_sub(1);
            continue;
        }
        uint64_t rv = s.resv.load(), n, at;
        bool full = false;
        for (;;) {
            n = rv >> 40;
            at = rv & kBytesMask;
            if (n + 1 > s.cap_n || at + len > s.cap_bytes) {
                full = true;
                break;
            }
            if (s.resv.compare_exchange_weak(rv, (n + 1) << 40 | (at + len))) break;
        }
        if (full) {
            s.writers.fetch_sub(1);
            b->Wake();
            if (++tries > 1000) return -2;  // both flushers busy and the open slot full: backpressure
            std::this_thread::yield();
            continue;
        }
        if (n == 0) s.first_ns.store(now_ns());
        s.off[n] = at;
        s.len[n] = len;
        s.conn[n] = conn;
        s.fn[n] = done;
        s.ctx[n] = ctx;
        memcpy(s.arena + at, req, len);
        s.writers.fetch_sub(1);
        b->n_submitted.fetch_add(1);
        if (n == 0 || n + 1 == b->max_n) b->Wake();
        return 0;
    }
}

int l7g_batcher_flush(l7g_batcher *b) {
    if (b->IsFlusher()) return -1;  // from a callback: it would wait on itself
    const uint64_t target = b->n_submitted.load();
    std::unique_lock<std::mutex> lk(b->mu);
    b->flush_gen++;
    b->cv.notify_all();
    b->done_cv.wait(lk, [&] { return b->completed >= target; });
    return 0;
}

void l7g_batcher_destroy(l7g_batcher *b) {
    if (!b || b->IsFlusher()) return;  // (from a callback: not allowed, see the header)
    b->stop.store(true);
    b->Wake();
    for (auto &t : b->th) t.join();
    FreeSlots(b);
    delete b;
}

void l7g_batcher_stats(l7g_batcher *b, uint64_t *requests, uint64_t *launches) {
    std::lock_guard<std::mutex> g(b->mu);
    if (requests) *requests = b->completed;
    if (launches) *launches = b->launches;
}

}  // extern "C"
