// Kafka correlation-ID rewriting of the in-agent Kafka proxy (product code,
// host side: it runs on the forwarding path, after the device verdicts).
//
//   pkg/kafka/correlation_cache.go:97-213   CorrelationCache: HandleRequest
//       gives every forwarded request the next sequence number (from 1) as its
//       correlation id and remembers the original; CorrelateResponse restores
//       the original id in the broker's response and forgets the entry; the
//       garbage collector drops entries older than RequestLifetime (5 min)
//   pkg/kafka/request.go:57-70     the request id: big-endian bytes 8..12
//   pkg/kafka/response.go:33-46    the response id: big-endian bytes 4..8
//   pkg/proxy/kafka.go:296-303,335,392  one cache per client connection;
//       allowed requests only (denied ones are answered by the proxy itself)
//
// The batch form rewrites the ids of a batch of forwarded frames in place,
// in batch order -- the order the reference's per-connection loop forwards
// them in.
#include <chrono>
#include <cstdint>
#include <mutex>
#include <unordered_map>

namespace {

struct Entry {
    uint32_t orig;
    std::chrono::steady_clock::time_point created;
};

uint32_t GetBE32(const uint8_t *p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }
void PutBE32(uint8_t *p, uint32_t v) {
    p[0] = (uint8_t)(v >> 24);
    p[1] = (uint8_t)(v >> 16);
    p[2] = (uint8_t)(v >> 8);
    p[3] = (uint8_t)v;
}

}  // namespace

struct l7g_kafka_corr {
    std::mutex mu;
    std::unordered_map<uint32_t, Entry> cache;
    uint32_t next = 1;  // nextSequenceNumber
    uint64_t expired = 0;
};

extern "C" {

l7g_kafka_corr *l7g_kafka_corr_create(void) { return new l7g_kafka_corr(); }

void l7g_kafka_corr_destroy(l7g_kafka_corr *c) { delete c; }

int l7g_kafka_corr_requests(l7g_kafka_corr *c, uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                            uint32_t *new_ids) {
    if (!c) return -1;
    std::lock_guard<std::mutex> g(c->mu);
    const auto now = std::chrono::steady_clock::now();
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *r = arena + off[i];
        const uint32_t orig = len[i] >= 12 ? GetBE32(r + 8) : 0;  // GetCorrelationID
        const uint32_t id = c->next++;
        if (len[i] >= 12) PutBE32(r + 8, id);  // SetCorrelationID
        c->cache[id] = Entry{orig, now};       // (an existing entry is overwritten, as there)
        if (new_ids) new_ids[i] = id;
    }
    return 0;
}

int l7g_kafka_corr_responses(l7g_kafka_corr *c, uint8_t *arena, const uint64_t *off, const uint32_t *len, uint32_t n,
                             uint8_t *found) {
    if (!c) return -1;
    std::lock_guard<std::mutex> g(c->mu);
    for (uint32_t i = 0; i < n; i++) {
        uint8_t *r = arena + off[i];
        const uint32_t id = len[i] >= 8 ? GetBE32(r + 4) : 0;
        auto it = c->cache.find(id);
        const bool hit = it != c->cache.end();
        if (hit) {
            if (len[i] >= 8) PutBE32(r + 4, it->second.orig);
            c->cache.erase(it);
        }
        if (found) found[i] = hit ? 1 : 0;
    }
    return 0;
}

uint64_t l7g_kafka_corr_gc(l7g_kafka_corr *c, uint64_t lifetime_ms) {
    if (!c) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    const auto cutoff = std::chrono::steady_clock::now() - std::chrono::milliseconds(lifetime_ms);
    uint64_t n = 0;
    for (auto it = c->cache.begin(); it != c->cache.end();) {
        if (it->second.created <= cutoff) {
            it = c->cache.erase(it);
            n++;
        } else {
            ++it;
        }
    }
    c->expired += n;
    return n;
}

uint64_t l7g_kafka_corr_size(l7g_kafka_corr *c) {
    if (!c) return 0;
    std::lock_guard<std::mutex> g(c->mu);
    return c->cache.size();
}

}  // extern "C"
