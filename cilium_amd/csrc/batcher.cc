// Asynchronous request batcher (product code, include/l7gpu.h l7g_batcher_*).
//
// Envoy's HTTP filter asks for one verdict per request from a worker's event
// loop (envoy/cilium_l7policy.cc:127-182).  One device launch per request is
// all latency and no throughput, so callers submit requests here instead and
// get a callback.  Layout (round 4):
//   * submitters write straight into a pinned batch slot, in the layout the
//     device copy reads (offsets, lengths, connections, request bytes): a
//     slot is cut into kLanes lanes (a range of entries and of request bytes
//     each, with its own reservation word on its own cache line; a thread
//     starts at its own lane and moves only to later ones), one fetch-and-add on a lane's word takes an
//     entry and a byte range, the submitting threads copy their bytes in
//     parallel, and a per-entry ready byte publishes it -- no lock, and one
//     atomic that the other threads seldom touch;
//   * kFlushers flusher threads each seal the open slot (once max_requests
//     are in it, its first request has waited max_wait_us, or a flush is asked
//     for): they open a free slot in its place, set the sealed bit of each of
//     the old one's lane words (which fixes its lanes' counts), wait for their
//     entries' ready bytes, close the lanes' entries up (16 bytes each) and
//     classify the slot where it lies -- the arrays in one copy, the lanes'
//     bytes in one 2-D copy (a small batch is packed and read in place
//     instead), one launch, no gather of request bytes on the host -- on the
//     flusher's own stream, then run its callbacks; so one batch is on the
//     device while the next fills;
//   * callbacks run on the flusher threads, batch after batch in the order
//     the slots were opened (a thread's requests in submission order); a
//     callback must not call l7g_batcher_flush or l7g_batcher_destroy (both
//     return at once, doing nothing, when called from a flusher thread);
//   * a slot holds 2 x max_requests requests (at least 1024) and 2 KiB of
//     request bytes per request; when both flushers are busy and every lane
//     of the open slot is full, submit returns -2 (backpressure) and the
//     caller answers the request itself.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/l7gpu.h"
#include "capi_internal.h"

namespace {

constexpr int kFlushers = 2;
constexpr int kSlots = kFlushers + 2;  // one per flusher, the open one, and one ready to open
constexpr int kLanes = 8;
// Lane::resv = sealed << 63 | count << 40 | lane arena bytes
constexpr uint64_t kSealed = 1ull << 63;
constexpr uint64_t kBytesMask = (1ull << 40) - 1;
constexpr uint64_t kOne = 1ull << 40;
constexpr uint32_t kMinSlotRequests = 1024;
constexpr uint32_t kMaxBatchRequests = 1u << 16;  // max_requests cap (slots of 2 x 64 Ki requests)
constexpr uint64_t kSlotBytesPerRequest = 2048;
constexpr int kSubmitTries = 1000;
constexpr uint32_t kPackMaxRequests = 256;     // a batch this small is packed and read in place
constexpr uint64_t kPackMaxBytes = 192 * 1024;
using Clock = std::chrono::steady_clock;
enum : uint8_t { EMPTY = 0, READY = 1, HOLE = 2 };  // Slot::ready
enum : int { FREE = 0, OPEN = 1, SEALED = 2 };

int64_t now_ns() { return Clock::now().time_since_epoch().count(); }
uint64_t Count(uint64_t rv) { return (rv & ~kSealed) >> 40; }

std::atomic<uint32_t> g_next_lane{0};
thread_local int t_lane = -1;  // the calling thread's home lane
// where the calling thread's last request went: its next one in the same slot
// goes to that lane or a later one, so that its requests stay in order
thread_local struct {
    const void *slot;
    uint64_t gen;
    int lane;
} t_last = {nullptr, 0, 0};

struct alignas(64) Lane {
    std::atomic<uint64_t> resv{0};
};

struct Slot {
    uint8_t *mem = nullptr;  // pinned; plain malloc only for a host-only engine (no device to copy to)
    bool pinned = false;
    uint64_t *off = nullptr;  // [cap_n], then len [cap_n], conn [cap_n]: lane l owns entries [l * ln, (l + 1) * ln)
    uint32_t *len = nullptr, *conn = nullptr;
    uint8_t *arena = nullptr;  // lane l owns bytes [l * lb, (l + 1) * lb)
    std::unique_ptr<std::atomic<uint8_t>[]> ready;
    std::vector<l7g_done_fn> fn;
    std::vector<void *> ctx;
    uint32_t cap_n = 0, ln = 0;
    uint64_t lb = 0;
    uint64_t gen = 0;  // 1, 2, ...: the order slots are opened, sealed and answered in
    Lane lane[kLanes];
    alignas(64) std::atomic<int64_t> first_ns{0};  // when its first request was reserved
    std::atomic<bool> full{false};                  // a submitter found no room: seal it now
    std::atomic<int> state{FREE};

    uint32_t Count() const {  // requests reserved so far
        uint32_t c = 0;
        for (const auto &l : lane) c += (uint32_t)std::min<uint64_t>(::Count(l.resv.load(std::memory_order_relaxed)), ln);
        return c;
    }
};

}  // namespace

struct l7g_batcher {
    l7g_engine *e = nullptr;
    uint32_t max_n = 1;
    std::chrono::microseconds max_wait{0};
    Slot slots[kSlots];
    std::atomic<int> open_idx{0};
    std::atomic<bool> stop{false};
    // flusher coordination
    std::mutex mu;
    std::condition_variable cv, done_cv;
    uint64_t flush_gen = 0;                // a flush was asked for: seal what is open at once
    uint64_t completed = 0, launches = 0;  // (under mu)
    uint64_t delivered = 0;                // slots answered, = the gen of the last one (under mu)
    uint64_t next_gen = 1;                 // (under seal_mu)
    std::atomic<uint64_t> t_ns[5] = {};    // l7g_batcher_timing
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
    uint32_t OpenCount() const { return slots[open_idx.load()].Count(); }

    // Seals the open slot if it holds requests and a free slot can take its
    // place; returns its index and its lanes' reservation words at the seal,
    // or -1.
    int Seal(uint64_t rv[kLanes]) {
        std::lock_guard<std::mutex> g(seal_mu);
        const int i = open_idx.load();
        Slot &s = slots[i];
        if (s.Count() == 0) return -1;
        int j = -1;
        for (int k = 1; k < kSlots && j < 0; k++)
            if (slots[(i + k) % kSlots].state.load() == FREE) j = (i + k) % kSlots;
        if (j < 0) return -1;  // (cannot happen with kSlots = kFlushers + 2; the open slot keeps filling)
        Slot &t = slots[j];
        t.gen = next_gen++;
        t.first_ns.store(0);
        t.full.store(false);
        for (auto &l : t.lane) l.resv.store(0);
        t.state.store(OPEN);
        open_idx.store(j);
        s.state.store(SEALED);
        // a submitter's fetch-and-add lands either before this (its entry is
        // counted and waited for) or after it (it sees the bit and moves on)
        for (int l = 0; l < kLanes; l++) rv[l] = s.lane[l].resv.fetch_or(kSealed);
        return i;
    }

    // Waits for the sealed slot's entries, closes them up to [0, n) (16-byte
    // entries; holes and the gaps between lanes dropped) and describes its
    // request bytes: a small batch is packed into one piece (read in place),
    // a larger one is the lanes as rows of one 2-D copy (each row as wide as
    // the fullest lane; a thread fills its lane before moving to the next, so
    // the rows are close to full).  The offsets are rebased onto what the
    // device will see.  Returns n.
    uint32_t Gather(Slot &s, const uint64_t rv[kLanes], l7g_host_seg *seg) {
        uint32_t cnt[kLanes], total = 0;
        uint64_t used[kLanes], bytes = 0, width = 0;
        int rows = 0;
        for (int l = 0; l < kLanes; l++) {
            cnt[l] = (uint32_t)std::min<uint64_t>(Count(rv[l]), s.ln);
            used[l] = std::min<uint64_t>(rv[l] & kBytesMask, s.lb);
            total += cnt[l];
            bytes += used[l];
            width = std::max(width, used[l]);
            if (used[l] || cnt[l]) rows = l + 1;  // (a lane of zero-length requests still needs its row in range)
        }
        const bool pack = total <= kPackMaxRequests && bytes <= kPackMaxBytes;
        width = (width + 15) & ~(uint64_t)15;  // (rows start 16-byte aligned on the device too)
        if (width > s.lb) width = s.lb;
        uint32_t m = 0;
        uint64_t at = 0;
        for (int l = 0; l < kLanes; l++) {
            const uint32_t e0 = (uint32_t)l * s.ln;
            const uint64_t b0 = (uint64_t)l * s.lb;
            const uint64_t dst = pack ? at : (uint64_t)l * width;
            for (uint32_t k = e0; k < e0 + cnt[l]; k++) {
                uint8_t st;
                while ((st = s.ready[k].load(std::memory_order_acquire)) == EMPTY) std::this_thread::yield();
                s.ready[k].store(EMPTY, std::memory_order_relaxed);
                if (st == HOLE) continue;  // reserved, but its bytes did not fit the lane
                s.off[m] = s.off[k] - b0 + dst;
                s.len[m] = s.len[k];
                s.conn[m] = s.conn[k];
                s.fn[m] = s.fn[k];
                s.ctx[m] = s.ctx[k];
                m++;
            }
            if (pack && used[l]) {
                memmove(s.arena + at, s.arena + b0, used[l]);  // (at <= b0)
                at += used[l];
            }
        }
        if (pack) *seg = {s.arena, at, at, 1};
        else *seg = {s.arena, width, s.lb, (uint32_t)rows};
        return m;
    }

    void Run() {
        std::vector<uint8_t> v;
        std::vector<int32_t> r;
        std::vector<uint32_t> c;
        l7g_host_seg seg;
        // this thread's stream and staging, made now for the largest batch a
        // slot can hold rather than grown under load
        l7g_host_reserve(e, slots[0].cap_n, slots[0].lb * kLanes);
        uint64_t seen_flush = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(mu);
                for (;;) {
                    const uint32_t p = OpenCount();
                    if (stop && p == 0) return;
                    if (p >= max_n || (p && (stop || flush_gen != seen_flush || slots[open_idx.load()].full.load())))
                        break;
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
            uint64_t rv[kLanes];
            const int i = Seal(rv);
            if (i < 0) {  // the other flusher sealed it first
                std::this_thread::yield();
                continue;
            }
            Slot &s = slots[i];
            const uint64_t gen = s.gen;  // (read now: once the slot is FREE, a Seal may reopen it under a new gen)
            const int64_t t0 = now_ns();
            const uint32_t n = Gather(s, rv, &seg);
            v.resize(n);
            r.resize(n);
            c.resize(n);
            const int64_t t1 = now_ns();
            const int rc = l7g_host_run_pinned(e, n, s.off, s.cap_n, &seg, 1, v.data(), r.data(), c.data());
            const int64_t t2 = now_ns();
            {  // callbacks in the order the slots were opened
                std::unique_lock<std::mutex> lk(mu);
                done_cv.wait(lk, [&] { return delivered + 1 == gen; });
            }
            const int64_t t3 = now_ns();
            for (uint32_t k = 0; k < n; k++) {
                if (rc != 0) s.fn[k](s.ctx[k], L7G_UNSUPPORTED, -1, 0);
                else s.fn[k](s.ctx[k], v[k], r[k], c[k]);
            }
            s.state.store(FREE);
            const int64_t t4 = now_ns();
            t_ns[0] += (uint64_t)(t1 - t0);
            t_ns[1] += (uint64_t)(t2 - t1);
            t_ns[3] += (uint64_t)(t3 - t2);
            t_ns[2] += (uint64_t)(t4 - t3);
            for (uint64_t m = t_ns[4].load(); n > m && !t_ns[4].compare_exchange_weak(m, n);) {
            }
            {
                std::lock_guard<std::mutex> g(mu);
                delivered = gen;
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
    // (capped so that the four pinned slots stay within what a host can pin: 4 x 128 Ki x 2 KiB = 1 GiB)
    b->max_n = std::min<uint32_t>(max_requests ? max_requests : 1, kMaxBatchRequests);
    b->max_wait = std::chrono::microseconds(max_wait_us);
    const uint32_t cap_n = (std::max<uint32_t>(2 * b->max_n, kMinSlotRequests) + kLanes - 1) / kLanes * kLanes;
    const uint64_t cap_bytes = (uint64_t)cap_n * kSlotBytesPerRequest;
    const size_t meta = ((size_t)cap_n * 16 + 255) & ~(size_t)255;
    const size_t total = meta + cap_bytes + 64;  // (+64: aligned 16-byte reads past the last request stay inside)
    for (auto &s : b->slots) {
        s.mem = (uint8_t *)l7g_pinned_alloc(total);
        s.pinned = s.mem != nullptr;
        // the device path reads a small batch in place (zero copy) and copies a
        // large one with a 2-D copy: both need pinned memory, so an engine with
        // a device gets no batcher rather than one that answers UNSUPPORTED
        if (!s.mem && !l7g_engine_has_device(e)) s.mem = (uint8_t *)malloc(total);
        if (!s.mem) {
            FreeSlots(b);
            delete b;
            return nullptr;
        }
        s.off = (uint64_t *)s.mem;
        s.len = (uint32_t *)(s.mem + (size_t)cap_n * 8);
        s.conn = (uint32_t *)(s.mem + (size_t)cap_n * 12);
        s.arena = s.mem + meta;
        s.ready.reset(new std::atomic<uint8_t>[cap_n]);
        for (uint32_t k = 0; k < cap_n; k++) s.ready[k].store(EMPTY, std::memory_order_relaxed);
        s.fn.resize(cap_n);
        s.ctx.resize(cap_n);
        s.cap_n = cap_n;
        s.ln = cap_n / kLanes;
        s.lb = cap_bytes / kLanes;
    }
    b->slots[0].gen = b->next_gen++;
    b->slots[0].state.store(OPEN);
    for (auto &t : b->th) t = std::thread([b] { b->Run(); });
    return b;
}

uint32_t l7g_batcher_max_requests(const l7g_batcher *b) { return b ? b->max_n : 0; }

int l7g_batcher_submit(l7g_batcher *b, const uint8_t *req, uint32_t len, uint32_t conn, l7g_done_fn done, void *ctx) {
    if (b->stop.load(std::memory_order_relaxed)) return -1;  // (a submit racing destroy is the caller's error)
    if (len > b->slots[0].lb) return -2;                       // never fits a lane
    if (t_lane < 0) t_lane = (int)(g_next_lane.fetch_add(1) % kLanes);
    int tries = 0;
    for (;;) {
        Slot &s = b->slots[b->open_idx.load()];
        // this thread's lane first, then the ones after it.  A thread that
        // already has entries in this slot never goes back (its requests stay
        // in submission order when the lanes are closed up); one with none in
        // it yet wraps round to the lanes before its own, so a lone submitter
        // can fill the whole slot whichever lane is its home.
        const bool fresh = !(t_last.slot == &s && t_last.gen == s.gen);
        const int l0 = fresh ? t_lane : t_last.lane;
        const int nl = fresh ? kLanes : kLanes - l0;
        int l = l0;
        uint64_t rv = 0;
        bool sealed = false, got = false;
        for (int step = 0; step < nl; step++) {
            l = (l0 + step) % kLanes;
            Lane &ln = s.lane[l];
            const uint64_t cur = ln.resv.load(std::memory_order_relaxed);
            if (cur & kSealed) {
                sealed = true;  // sealed under us: the next slot is already open
                break;
            }
            // (checked before adding, so a full lane's count grows by at most one per thread)
            if (Count(cur) >= s.ln || (cur & kBytesMask) + len > s.lb) continue;
            rv = ln.resv.fetch_add(kOne | len);
            if (rv & kSealed) {
                sealed = true;
                break;
            }
            const uint64_t n = Count(rv);
            if (n >= s.ln) continue;  // filled under us: no entry to publish
            if ((rv & kBytesMask) + len > s.lb) {  // an entry, but no room for its bytes: leave a hole
                s.ready[(size_t)l * s.ln + n].store(HOLE, std::memory_order_release);
                continue;
            }
            got = true;
            break;
        }
        if (sealed) continue;
        if (!got) {  // no room for this thread: have the slot sealed
            s.full.store(true);
            b->Wake();
            if (++tries > kSubmitTries) return -2;  // both flushers busy: backpressure
            std::this_thread::yield();
            continue;
        }
        t_last = {&s, s.gen, l};
        const uint64_t n = Count(rv), at = (uint64_t)l * s.lb + (rv & kBytesMask);
        const size_t x = (size_t)l * s.ln + n;
        int64_t z = 0;
        const bool first = n == 0 && s.first_ns.load(std::memory_order_relaxed) == 0 &&
                           s.first_ns.compare_exchange_strong(z, now_ns());
        s.off[x] = at;
        s.len[x] = len;
        s.conn[x] = conn;
        s.fn[x] = done;
        s.ctx[x] = ctx;
        memcpy(s.arena + at, req, len);
        s.ready[x].store(READY, std::memory_order_release);
        // wake a flusher to start the batch's clock, and now and then to count it
        if (first || (n + 1) % std::max<uint32_t>(b->max_n / kLanes, 1) == 0) b->Wake();
        return 0;
    }
}

int l7g_batcher_flush(l7g_batcher *b) {
    if (b->IsFlusher()) return -1;  // from a callback: it would wait on itself
    uint64_t target;
    {  // every request submitted before this call is in the open slot or an earlier one
        std::lock_guard<std::mutex> g(b->seal_mu);
        const Slot &s = b->slots[b->open_idx.load()];
        target = s.Count() ? s.gen : s.gen - 1;
    }
    std::unique_lock<std::mutex> lk(b->mu);
    b->flush_gen++;
    b->cv.notify_all();
    b->done_cv.wait(lk, [&] { return b->delivered >= target; });
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

void l7g_batcher_timing(l7g_batcher *b, uint64_t out[5]) {
    for (int k = 0; k < 5; k++) out[k] = b->t_ns[k].load();
}

void l7g_batcher_stats(l7g_batcher *b, uint64_t *requests, uint64_t *launches) {
    std::lock_guard<std::mutex> g(b->mu);
    if (requests) *requests = b->completed;
    if (launches) *launches = b->launches;
}

}  // extern "C"
