// Kafka request classification on gfx950 (product code).
//
// One lane per request frame.  Each lane restates, sequentially over its own
// bytes, the reference's decode path: proto.ReadReq framing
// (vendor/github.com/optiopay/kafka/proto/messages.go:124-165), the typed
// decoders (:504-537, :767-824, :1033-1054, :1173-1228, :1389-1430,
// :1591-1647, :1810-1858) with io.ReadFull / LimitReader semantics
// (serialization.go:19-203), readMessageSet with CRC32-IEEE per message and
// stop-without-drain (:363-494), then MatchesRule (pkg/kafka/policy.go:200-225)
// against the connection's rule set using the precomputed topic / key views
// (engine/kafka_compile.h).  Requests with compressed messages are listed for
// kafka_inflate_kernel (kafka_inflate.hip), which decodes them.
//
// Memory layout of the walk (round 4).  Every lane owns a window of kWin
// 16-byte chunks of its request in LDS: chunk k of the request (k counted from
// the 16-byte aligned address that holds its first byte) lives in slot
// k % kWin, at slot * 1 KiB + 16 * lane of the wave's window area, so every
// window read is one conflict-free ds_read_b128 whatever chunk each lane reads.
// The wave works in rounds: the windows move (LDS-DMA of the chunks each lane
// is missing, global_load_lds_dwordx4, one instruction per slot), then every
// lane decodes from its window until it needs a byte outside it.  So each
// request byte crosses HBM once, in whole 16-byte pieces, and the decoders'
// dependent reads are LDS round trips instead of L2 / HBM ones (round 3 read
// through a per-lane register cursor and moved 2.9x the request bytes: lines
// left L2 between a lane's touches).
//
// Produce requests -- nearly all of the bytes -- are decoded by a resumable
// step machine (header, topic, partition, message header, CRC segment), so a
// lane can stop at a window edge and resume in the next round.  A step reads
// only resident chunks; one that runs past the window is rolled back and
// retried after the window moved to its start, and one that is longer than a
// window (a topic name over ~240 bytes, say) reads its bytes from HBM.  The
// other kinds are short (their first window holds them) and run the
// lane-serial decoders in one step, any byte outside the window read from HBM.
// A lane that finishes takes the wave's next list entry at once, so lanes do
// not idle while the longest request of a group finishes.
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "kafka_dec.h"

namespace l7 {

namespace {

#ifndef L7G_KAFKA_WIN  // window chunks (16 B) per lane, a multiple of 4
#define L7G_KAFKA_WIN 16
#endif
#ifndef L7G_KAFKA_BWAVES  // waves per workgroup (the CRC tables are shared by its waves)
#define L7G_KAFKA_BWAVES 4
#endif
constexpr uint32_t kWin = L7G_KAFKA_WIN;
constexpr int kWaves = L7G_KAFKA_BWAVES;
constexpr int kBlock = 64 * kWaves;
static_assert(kWin >= 8 && kWin % 4 == 0 && (kWin & (kWin - 1)) == 0, "window: a power of two >= 8");
constexpr uint32_t kNoWin = 0x80000000u;  // w0 of a lane without a window
constexpr uint32_t kNoChunk = 0xFFFFFFFFu;

typedef __attribute__((address_space(3))) const gm_u32x4 lds_u32x4;

__device__ __forceinline__ uint4 lds_read16(uint32_t a) {
    const gm_u32x4 v = *(lds_u32x4 *)(size_t)a;
    return make_uint4(v.x, v.y, v.z, v.w);
}

// ---- the per-lane window cursor
struct WCur {
    uint64_t ab;   // 16-byte aligned address of the chunk holding the request's first byte
    uint32_t a0;   // request start within that chunk
    uint32_t w0;   // first resident chunk (kNoWin: none)
    uint32_t lds;  // LDS address of this lane's slot 0
    uint32_t ck;   // chunk held in x0..x3 (kNoChunk: none)
    uint32_t x0, x1, x2, x3;
    uint32_t gok;   // a chunk outside the window is read from HBM (else: miss)
    uint32_t miss;  // a read missed the window (the step is rolled back)
};

__device__ __forceinline__ bool w_res(const WCur &w, uint32_t k) { return k - w.w0 < kWin; }

__device__ __forceinline__ void w_fill(WCur &w, uint32_t k) {
    if (k == w.ck) return;
    uint4 v;
    if (w_res(w, k)) {
        v = lds_read16(w.lds + (k & (kWin - 1)) * 1024u);
    } else if (w.gok) {
        v = gload16(w.ab + 16ull * k);
    } else {
        w.miss = 1;
        w.ck = kNoChunk;
        w.x0 = w.x1 = w.x2 = w.x3 = 0;
        return;
    }
    w.x0 = v.x; w.x1 = v.y; w.x2 = v.z; w.x3 = v.w;
    w.ck = k;
}
// little-endian bytes j .. j+3 of the held chunk (j <= 12)
__device__ __forceinline__ uint32_t w_word_at(const WCur &w, uint32_t j) {
    const uint32_t a = w.x0, b = w.x1, c = w.x2, d = w.x3;
    const uint32_t i = j >> 2;
    const uint32_t lo = i == 0 ? a : i == 1 ? b : i == 2 ? c : d;
    const uint32_t hi = i == 0 ? b : i == 1 ? c : i == 2 ? d : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, j & 3);
}
__device__ __forceinline__ uint32_t w_byte(WCur &w, uint32_t pos) {
    const uint32_t a = w.a0 + pos;
    w_fill(w, a >> 4);
    return w_word_at(w, a & 12) >> ((a & 3) * 8) & 0xFFu;
}
// big-endian n-byte field at request position pos (n = 1, 2, 4)
__device__ __forceinline__ uint32_t w_be(WCur &w, uint32_t pos, int n) {
    const uint32_t a = w.a0 + pos;
    const uint32_t j = a & 15;
    if (j + (uint32_t)n <= 16) {
        w_fill(w, a >> 4);
        const uint32_t v = bswap32(w_word_at(w, j));
        return n == 4 ? v : v >> (32 - 8 * n);
    }
    uint32_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | w_byte(w, pos + i);
    return v;
}
// 4 bytes at pos as a little-endian word
__device__ __forceinline__ uint32_t w_le4(WCur &w, uint32_t pos) {
    const uint32_t a = w.a0 + pos;
    const uint32_t j = a & 15;
    if (j <= 12) {
        w_fill(w, a >> 4);
        return w_word_at(w, j);
    }
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) v |= w_byte(w, pos + i) << (8 * i);
    return v;
}

// ---- io.ReadFull / LimitReader decoding over request positions (serialization.go:19-203)
struct KD {
    uint32_t pos, end;
    int32_t limit;  // LimitReader remaining, -1 = none
    int err;        // 0 ok, 1 EOF, 2 ErrUnexpectedEOF, 3 other
};
__device__ __forceinline__ uint32_t kd_avail(const KD &d) {
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint32_t)d.limit < a) a = (uint32_t)d.limit;
    return a;
}
__device__ __forceinline__ uint32_t kd_read(KD &d, uint32_t n) {
    const uint32_t at = d.pos;
    if (n == 0) return at;
    const uint32_t a = kd_avail(d);
    if (a == 0) { d.err = 1; return at; }
    const uint32_t take = a < n ? a : n;
    d.pos += take;
    if (d.limit >= 0) d.limit -= (int32_t)take;
    if (take < n) d.err = 2;
    return at;
}
__device__ __forceinline__ int32_t kd_int(WCur &w, KD &d, int n) {
    if (d.err) return 0;
    const uint32_t at = kd_read(d, (uint32_t)n);
    if (d.err) return 0;
    const uint32_t v = w_be(w, at, n);
    return n == 1 ? (int32_t)(int8_t)v : n == 2 ? (int32_t)(int16_t)v : (int32_t)v;
}
__device__ __forceinline__ void kd_skip(KD &d, int n) {
    if (d.err) return;
    kd_read(d, (uint32_t)n);
}
// DecodeString -> (off, len); len < 1 => ""
__device__ __forceinline__ void kd_string(WCur &w, KD &d, uint32_t &off, uint32_t &len) {
    off = 0; len = 0;
    if (d.err) return;
    const int16_t sl = (int16_t)kd_int(w, d, 2);
    if (d.err || sl < 1) return;
    const uint32_t at = kd_read(d, (uint32_t)sl);
    if (d.err) return;
    off = at; len = (uint32_t)sl;
}
// DecodeArrayLen(nullable): -1 null; sets bad on ErrInvalidArrayLen
__device__ __forceinline__ int32_t kd_arraylen(WCur &w, KD &d, bool nullable, bool &bad) {
    const int32_t l = kd_int(w, d, 4);
    bad = false;
    if (l < 0) { if (nullable) return -1; bad = true; return 0; }
    if ((uint32_t)l > kMaxParseBuf) { bad = true; return 0; }
    return l;
}
__device__ __forceinline__ void kd_bytes(WCur &w, KD &d) {
    if (d.err) return;
    const int32_t sl = kd_int(w, d, 4);
    if (d.err || sl < 1) return;
    if ((uint32_t)sl > kMaxParseBuf) { d.err = 3; return; }
    kd_read(d, (uint32_t)sl);
}

// Interned id of the request string [s, s + n) (topic or client id), -1 if
// the rule tables do not know it: word hash (l7_whash_*), linear probing,
// then a word-wise compare: the first 16 bytes against the slot's copy (the
// words were read for the hash), the rest against the 4-byte aligned,
// zero-padded table string.
__device__ __forceinline__ int32_t str_lookup(const DevStrSlot *tab, uint32_t mask, const uint8_t *strings, WCur &w,
                                              uint32_t s, uint32_t n) {
#ifdef KEXP_NOLOOKUP
    return -1;
#endif
    uint32_t h = kWHashSeed;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;  // the first 16 bytes, zero-padded
    for (uint32_t i = 0; i < n; i += 4) {
        const uint32_t r = n - i;
        const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u;
        const uint32_t x = w_le4(w, s + i) & keep;
        h = l7_whash_step(h, x);
        p0 = i == 0 ? x : p0;
        p1 = i == 4 ? x : p1;
        p2 = i == 8 ? x : p2;
        p3 = i == 12 ? x : p3;
    }
    if (w.miss) return -1;  // the step is rolled back
    h = l7_whash_final(h, n);
    for (uint32_t slot = h & mask;; slot = (slot + 1) & mask) {
        const DevStrSlot e = tab[slot];
        if (!e.used) return -1;
        if (e.hash == h && e.len == n) {
            bool eq = e.pre[0] == p0 && e.pre[1] == p1 && e.pre[2] == p2 && e.pre[3] == p3;
            const uint32_t *t = reinterpret_cast<const uint32_t *>(strings + e.str_off);
            for (uint32_t i = 16; i < n && eq && !w.miss; i += 4) {
                const uint32_t r = n - i;
                const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u;
                eq = t[i >> 2] == (w_le4(w, s + i) & keep);
            }
            if (eq) return e.id;
        }
    }
}

__device__ __forceinline__ bool is_topic_api_key(int k) {
    // 0 1 2 3 4 5 6 8 9 19 20 21 23 24 27 28 34 35 37
    if (k < 0 || k > 37) return false;
    const uint64_t m = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 4) | (1ull << 5) | (1ull << 6) |
                       (1ull << 8) | (1ull << 9) | (1ull << 19) | (1ull << 20) | (1ull << 21) | (1ull << 23) |
                       (1ull << 24) | (1ull << 27) | (1ull << 28) | (1ull << 34) | (1ull << 35) | (1ull << 37);
    return (m >> k) & 1;
}

struct ReqInfo {
    int kind;
    int version;
    int typed;      // 0 nil request, 1 typed with topics/ClientID, 2 ConsumerMetadata
    int32_t client; // interned id, -2 unknown / empty
};

__device__ __forceinline__ bool rule_matches(const DevKafkaRule &r, const ReqInfo &q) {
    if (!r.any_key && (q.kind < 0 || q.kind > 63 || !((r.keymask >> q.kind) & 1))) return false;
    if (r.has_version && r.version != q.version) return false;
    if (!r.has_topic && r.client < 0) return true;
    if (q.typed == 1) return r.client < 0 || r.client == q.client;
    if (q.typed == 2) return true;
    return !(r.has_topic && is_topic_api_key(q.kind));
}

// first position of topic `tid`'s rule list that matches, kInf if none
__device__ __forceinline__ uint32_t topic_first(const KafkaTables &T, const DevKafkaRuleset &rs, const ReqInfo &q, int32_t tid) {
    if (tid < 0 || rs.ntopics == 0) return kInf;
    uint32_t off, cnt;
    if (rs.tdense_off != ~0u) {
        const uint4 *ep = reinterpret_cast<const uint4 *>(T.index + rs.tdense_off +
                                                          (uint32_t)(sizeof(DevKafkaTopicEnt) / 4) * (uint32_t)tid);
        const uint4 e0 = ep[0], e1 = ep[1], e2 = ep[2];
        off = e0.y;
        cnt = e0.z;
        if (cnt == 0) return kInf;
        DevKafkaRule r0;
        const uint32_t wd[6] = {e1.x, e1.y, e1.z, e1.w, e2.x, e2.y};
        __builtin_memcpy(&r0, wd, sizeof r0);
        if (rule_matches(r0, q)) return e0.x;
        for (uint32_t i = 1; i < cnt; i++) {
            uint32_t p = T.index[off + i];
            if (rule_matches(T.rules[rs.rule_first + p], q)) return p;
        }
        return kInf;
    } else {
        const uint32_t *dir = T.index + rs.topics_off;
        uint32_t lo = 0, hi = rs.ntopics;
        while (lo < hi) {
            uint32_t m = (lo + hi) >> 1;
            if (dir[3 * m] < (uint32_t)tid) lo = m + 1; else hi = m;
        }
        if (lo >= rs.ntopics || dir[3 * lo] != (uint32_t)tid) return kInf;
        off = dir[3 * lo + 1];
        cnt = dir[3 * lo + 2];
    }
    for (uint32_t i = 0; i < cnt; i++) {
        uint32_t p = T.index[off + i];
        if (rule_matches(T.rules[rs.rule_first + p], q)) return p;
    }
    return kInf;
}

// MatchesRule's rule choice (pkg/kafka/policy.go:200-225): the first rule in
// evaluation order that holds, as a position; ntopics / cmax from the walk
// (cmax: over the topics, the largest first-matching position).
__device__ __forceinline__ uint32_t match_rules(const KafkaTables &T, const DevKafkaRuleset &rs, const ReqInfo &q,
                                                uint32_t ntopics, uint32_t cmax) {
    uint32_t best = kInf;
    if (ntopics == 0) {
        const int key = (q.kind >= 0 && q.kind < 64) ? q.kind : 64;
        const uint32_t off = T.index[rs.bykey_off + 2 * key], cnt = T.index[rs.bykey_off + 2 * key + 1];
        for (uint32_t i = 0; i < cnt; i++) {
            const uint32_t pp = T.index[off + i];
            if (rule_matches(T.rules[rs.rule_first + pp], q)) { best = pp; break; }
        }
    } else {
        for (uint32_t i = 0; i < rs.ntopicless; i++) {
            const uint32_t pp = T.index[rs.topicless_off + i];
            if (pp >= cmax) break;  // cannot beat topic completion
            if (rule_matches(T.rules[rs.rule_first + pp], q)) { best = pp; break; }
        }
        if (best == kInf) best = cmax;
    }
    return best;
}

// CRC32-IEEE of n bytes at byte j of the held chunk (j + n <= 16): 8-, 4- and
// <= 3-byte slicing steps, each step's lookups in flight together
__device__ __forceinline__ uint32_t crc_in_chunk(uint32_t tabaddr, const WCur &w, uint32_t c, uint32_t j, uint32_t n) {
    uint32_t i = 0;
    if (n >= 8) {
        c = crc_step8(tabaddr, w_word_at(w, j) ^ c, w_word_at(w, j + 4));
        i = 8;
    }
    if (n - i >= 4) {
        c = crc_step4(tabaddr, w_word_at(w, j + i) ^ c);
        i += 4;
    }
    if (i < n) c = crc_bytes3(tabaddr, c, w_word_at(w, j + i), n - i);
    return c;
}

// lane states
enum : uint32_t { ST_IDLE = 0, ST_START, ST_TOPIC, ST_PART, ST_MSG, ST_CRC, ST_NEW, ST_FIN };

// The decode of a non-produce request (typed kinds 1, 2, 3, 8, 9, 10 and the
// untyped ones), lane-serial over the window cursor.  Returns rc (0 ok, -1
// decode error), the raw topic count and the first matching rule position
// over the topics (messages.go decoders; MatchesRule's topic part).
__device__ __forceinline__ int decode_other(WCur &w, const KafkaTables &T, const DevKafkaRuleset &rs, ReqInfo &q, uint32_t rawlen,
                            uint32_t &ntopics, uint32_t &cmax) {
    KD d{0, rawlen, -1, 0};
    bool bad = false;
    kd_skip(d, 4); kd_skip(d, 2);
    const int16_t ver = (int16_t)kd_int(w, d, 2);
    kd_skip(d, 4);
    uint32_t co, cl;
    kd_string(w, d, co, cl);
    if (!d.err && cl > 0) q.client = str_lookup(T.client_hash, T.client_mask, T.strings, w, co, cl);
    if (q.client < 0) q.client = -2;
    const bool topics_on = q.typed == 1;
    int rc = 0;
    auto on_topic = [&](uint32_t to, uint32_t tl) {
        if (!topics_on) return;
        ntopics++;
        const int32_t tid = tl > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, w, to, tl) : -1;
        const uint32_t e = topic_first(T, rs, q, tid);
        cmax = cmax > e ? cmax : e;
    };
    int32_t nt, np;
    uint32_t o, l;
    switch (q.kind) {
    case 1:  // Fetch
        kd_skip(d, 4); kd_skip(d, 4); kd_skip(d, 4);
        if (ver >= 3) kd_skip(d, 4);
        if (ver >= 4) kd_skip(d, 1);
        nt = kd_arraylen(w, d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(w, d, o, l);
            on_topic(o, l);
            np = kd_arraylen(w, d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np && !d.err; p++) {
                kd_skip(d, 4); kd_skip(d, 8);
                if (ver >= 5) kd_skip(d, 8);
                kd_skip(d, 4);
            }
        }
        break;
    case 2:  // Offset
        kd_skip(d, 4);
        if (ver >= 2) kd_skip(d, 1);
        nt = kd_arraylen(w, d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(w, d, o, l);
            on_topic(o, l);
            np = kd_arraylen(w, d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np && !d.err; p++) {
                kd_skip(d, 4); kd_skip(d, 8);
                if (ver == 0) kd_skip(d, 4);
            }
        }
        break;
    case 3:  // Metadata
        nt = kd_arraylen(w, d, true, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) { kd_string(w, d, o, l); if (!d.err) on_topic(o, l); }
        if (ver >= 4) kd_skip(d, 1);
        break;
    case 8:  // OffsetCommit
        kd_string(w, d, o, l);
        if (ver >= 1) { kd_skip(d, 4); kd_string(w, d, o, l); }
        if (ver >= 2) kd_skip(d, 8);
        nt = kd_arraylen(w, d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(w, d, o, l);
            on_topic(o, l);
            np = kd_arraylen(w, d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np && !d.err; p++) {
                kd_skip(d, 4); kd_skip(d, 8);
                if (ver == 1) kd_skip(d, 8);
                uint32_t o2, l2;
                kd_string(w, d, o2, l2);
            }
        }
        break;
    case 9:  // OffsetFetch
        kd_string(w, d, o, l);
        nt = kd_arraylen(w, d, true, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(w, d, o, l);
            on_topic(o, l);
            np = kd_arraylen(w, d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np && !d.err; p++) kd_skip(d, 4);
        }
        break;
    case 10:  // ConsumerMetadata
        kd_string(w, d, o, l);
        if (ver >= 1) kd_skip(d, 1);
        break;
    }
    if (rc == 0 && d.err) rc = -1;
    return rc;
}

}  // namespace

// Two instantiations over partition_kernel's Kafka lists (L7_KAFKA_CLASSES
// kind / length classes, class c at sel + c * n, sel_count[c] entries each):
// kProduce walks the produce classes (2 .. kCls-1, longest first) with the
// resumable step machine; the other one walks fetch (class 0) and the other
// kinds (class 1), one step each.  Keeping them apart keeps each kernel's
// loop small (its code stays in the instruction cache) and its lanes on one
// kind of work.  work: a per-launch counter the launcher zeroes; waves take
// list entries 64 at a time from it.  answer_other: answer entries on
// connections that are not Kafka.
template <bool kProduce>
__global__ __launch_bounds__(kBlock) void kafka_classify_kernel(
    Batch B, KafkaTables T, const uint32_t *__restrict__ sel, const uint32_t *__restrict__ sel_count,
    uint32_t answer_other, uint32_t *__restrict__ zlist, uint32_t *__restrict__ zcount, uint32_t *__restrict__ work) {
    const uint32_t n = B.n, nconns = B.nconns;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    static_assert(kBlock >= 256, "one CRC table entry per thread");
    __shared__ uint32_t crctab[kProduce ? kCrcTables * 256 : 1];
    __shared__ __attribute__((aligned(16))) uint8_t winlds[kWaves][kWin * 1024];
    if (kProduce) crc_tables_init(crctab, threadIdx.x);
    const uint32_t tabaddr = (uint32_t)(uintptr_t)crctab;
    uint8_t *wwave = winlds[wave];
    constexpr int kCls = L7_KAFKA_CLASSES;
    static_assert(kCls == 8, "class 0 fetch, 1 other kinds, 2.. produce by length");
    constexpr int kLo = kProduce ? 2 : 0, kHi = kProduce ? kCls : 2;
    uint32_t kc[kCls];
    uint32_t m = 0;
#pragma unroll
    for (int c = 0; c < kCls; c++) {
        kc[c] = c >= kLo && c < kHi ? sel_count[c] : 0u;
        m += kc[c];
    }
    const uint64_t below = (1ull << lane) - 1;

    // ---- lane state
    uint32_t st = ST_IDLE;
    uint32_t idx = 0, rawlen = 0, last = 0;  // last: the request's last chunk
    int32_t rsi = 0;
    WCur w;
    w.ab = 0; w.a0 = 0; w.w0 = kNoWin; w.ck = kNoChunk; w.x0 = w.x1 = w.x2 = w.x3 = 0; w.gok = 0; w.miss = 0;
    w.lds = (uint32_t)(uintptr_t)wwave + 16u * lane;
    uint32_t blk = 0, bpos = 0;                    // blocked at request position bpos (window moves there)
    uint32_t pos = 0;                              // produce: the decoder position
    int32_t ver = 0, client = -2;
    int32_t nt = 0, t = 0, np = 0, p = 0, slimit = 0;
    uint32_t crcpos = 0, crcend = 0, crc = 0, crcst = 0, mflags = 0;
    uint32_t ntopics = 0, cmax = 0;
    uint32_t zflag = 0;
    uint8_t verdict = V_PARSE_ERROR;
    uint32_t consumed = 0;

    // ---- the wave's entry queue: qb = next unassigned entry of its current 64, qe = their end
    uint32_t qb = 0, qe = 0;

#ifdef KEXP_STATS
    uint32_t x_rounds = 0, x_iters = 0, x_done = 0;
    uint64_t x_tdma = 0, x_tproc = 0, x_tsetup = 0, x_t0 = 0;
    uint32_t x_steps[8] = {};
    uint32_t x_active = 0;
#endif
    for (uint32_t rounds = 0; rounds < (1u << 24); rounds++) {  // (a bound no launch reaches: every round makes progress)
#ifdef KEXP_STATS
        x_rounds++;
        if (x_t0) { const uint64_t t = clock64(); x_tproc += t - x_t0; x_t0 = t; }
#endif
        // 1. idle lanes take the next list entries
        {
            const uint64_t idle = __ballot(st == ST_IDLE);
            if (idle) {
                const uint32_t need = (uint32_t)__popcll(idle);
                const uint32_t rank = (uint32_t)__popcll(idle & below);
                const uint32_t have = qe - qb;
                uint32_t e1 = 0;  // entries from the current chunk, then from a new one
                if (need > have) {
                    uint32_t tk = 0;
                    if (lane == (uint32_t)__builtin_amdgcn_readfirstlane(lane)) tk = atomicAdd(work, 64u);
                    e1 = __builtin_amdgcn_readfirstlane(tk);
                }
                if (st == ST_IDLE) {
                    const uint32_t i = rank < have ? qb + rank : e1 + (rank - have);
                    st = i < m ? ST_NEW : ST_FIN;
                    if (i < m) {
                        // produce: the classes longest first (long requests start first)
                        uint32_t c = kProduce ? kHi - 1 : kLo, j = i;
#pragma unroll
                        for (int s = 0; s < kHi - kLo - 1; s++) {
                            const uint32_t cc = kProduce ? kHi - 1 - s : kLo + s;
                            if (c == cc && j >= kc[cc]) { j -= kc[cc]; c = kProduce ? cc - 1 : cc + 1; }
                        }
                        idx = sel[(size_t)c * n + j];
                    }
                }
                if (need > have) { qb = e1 + (need - have); qe = e1 + 64; }
                else qb += need;
            }
        }
        // 2. new lanes: connection, bounds, window origin
        if (st == ST_NEW) {
            const uint32_t ci = B.conn_ids[idx];
            const DevConn conn = ci < nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
            const uint64_t off = B.offs[idx];
            const uint32_t len = B.lens[idx];
            rsi = conn.ruleset;
            verdict = V_PARSE_ERROR; consumed = 0; zflag = 0; ntopics = 0; cmax = 0; client = -2;
            blk = 0; pos = 0;
            w.ab = (uint64_t)(uintptr_t)(B.arena + off) & ~15ull;
            w.a0 = (uint32_t)((uintptr_t)(B.arena + off) & 15);
            w.w0 = kNoWin; w.ck = kNoChunk; w.gok = 0;
            st = ST_START;
            bool ready = false;  // answered without decoding
            if (conn.proto != PROTO_KAFKA || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
                if (!answer_other || (L7_PROTO_OWNED(conn.proto) && conn.proto != PROTO_KAFKA)) {
                    st = ST_IDLE;  // another classifier's request
                } else {
                    verdict = V_UNSUPPORTED;  // unknown connection / no parser
                    ready = true;
                }
            } else if (!l7_in_arena(off, len, B.arena_len)) {
                verdict = V_UNSUPPORTED;  // out of contract
                ready = true;
            } else if (len < 6) {
                // ReadReq: fewer than 4 bytes, or a positive size with fewer than 6
                if (len < 4) verdict = V_INCOMPLETE;
                else {
                    uint32_t sz = 0;
                    for (uint32_t i = 0; i < 4; i++) sz = sz << 8 | B.arena[off + i];
                    verdict = (int32_t)sz <= 0 ? V_PARSE_ERROR : V_INCOMPLETE;
                }
                ready = true;
            }
            if (ready) {
                B.verdict[idx] = verdict;
                B.rule[idx] = -1;
                B.consumed[idx] = 0;
                st = ST_IDLE;
            } else if (st == ST_START) {
                last = (w.a0 + len - 1) >> 4;
                bpos = 0;
                blk = 1;  // the first window loads below
            }
        }
        if (__ballot(st != ST_FIN) == 0) break;
        // every lane answered at once: take more entries before moving windows
        if (__ballot(st != ST_IDLE && st != ST_FIN) == 0) continue;
        // 3. windows move: each blocked lane's window starts at the chunk of bpos;
        //    one LDS-DMA per slot for the lanes missing that slot's chunk
#ifdef KEXP_STATS
        { const uint64_t t = clock64(); x_tsetup += x_t0 ? t - x_t0 : 0; x_t0 = t;
          x_active += (uint32_t)__popcll(__ballot(st != ST_IDLE && st != ST_FIN)); }
#endif
        {
            const bool mv = blk != 0 && st != ST_IDLE && st != ST_FIN;
            const uint32_t nw = (w.a0 + bpos) >> 4;
#pragma unroll
            for (uint32_t s = 0; s < kWin; s++) {
                const uint32_t k = nw + ((s - nw) & (kWin - 1));
                const bool need = mv && k <= last && !w_res(w, k);
                if (need)
                    __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(w.ab + 16ull * k),
                                                     (__attribute__((address_space(3))) void *)(wwave + s * 1024), 16, 0,
                                                     0);
            }
            if (mv) { w.w0 = nw; blk = 0; }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
#ifdef KEXP_STATS
        { const uint64_t t = clock64(); x_tdma += t - x_t0; x_t0 = t; }
#endif
        // 4. every lane decodes from its window until it blocks or finishes
        for (;;) {
            const bool run = st >= ST_START && st <= ST_CRC && !blk;
            if (__ballot(run) == 0) break;
#ifdef KEXP_STATS
            x_iters++;
#endif
            if (!run) continue;
            const DevKafkaRuleset &rs = T.rulesets[rsi];
            bool done = false;
            int32_t rule_out = -1;
            w.miss = 0;
#ifdef KEXP_STATS
            x_steps[st & 7]++;
#endif
            const uint32_t spos = st == ST_CRC ? crcpos : pos;
            if (st == ST_START) {  // proto.ReadReq (messages.go:124-165), then the request header
                const int32_t size = (int32_t)w_be(w, 0, 4);
                const int16_t kind = (int16_t)w_be(w, 4, 2);
                const int16_t kver = (int16_t)w_be(w, 6, 2);
                const uint32_t len = B.lens[idx];
                done = true;
                if (size <= 0) verdict = V_PARSE_ERROR;
                else if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) verdict = V_PARSE_ERROR;
                else if ((uint32_t)size + 4 > len) verdict = V_INCOMPLETE;
                else if ((uint32_t)size + 4 < 12) verdict = V_PARSE_ERROR;
                else done = false;
                rawlen = (uint32_t)size + 4;
                if (!done && !kProduce) {
                    // fetch and the other kinds: one step, bytes outside the window from HBM
                    ReqInfo r;
                    r.kind = kind;
                    r.version = kver;
                    r.typed = (kind == 0 || kind == 1 || kind == 2 || kind == 3 || kind == 8 || kind == 9) ? 1
                            : (kind == 10 ? 2 : 0);
                    r.client = -2;
                    w.gok = 1;
                    uint32_t nt_ = 0, cm_ = 0;
                    int rc_ = 0;
                    if (r.typed) rc_ = decode_other(w, T, rs, r, rawlen, nt_, cm_);
                    done = true;
                    if (rc_ == 0) {  // ---- MatchesRule (pkg/kafka/policy.go:200-225)
                        consumed = rawlen;
                        verdict = V_DENY;
                        if (rs.any) {
                            const uint32_t best = match_rules(T, rs, r, nt_, cm_);
                            if (best != kInf) { verdict = V_ALLOW; rule_out = T.rules[rs.rule_first + best].gid; }
                        }
                    }
                } else if (!done) {
                    // Produce (messages.go:1591-1647): header fields up to the topic count
                    last = (w.a0 + rawlen - 1) >> 4;
                    KD d{0, rawlen, -1, 0};
                    bool bad = false;
                    kd_skip(d, 4); kd_skip(d, 2);
                    const int16_t v = (int16_t)kd_int(w, d, 2);
                    kd_skip(d, 4);
                    uint32_t co, cl;
                    kd_string(w, d, co, cl);
                    int32_t cid = -2;
                    if (!d.err && cl > 0) cid = str_lookup(T.client_hash, T.client_mask, T.strings, w, co, cl);
                    if (cid < 0) cid = -2;
                    uint32_t o, l;
                    if (v >= 3) kd_string(w, d, o, l);
                    kd_skip(d, 2); kd_skip(d, 4);
                    const int32_t ntp = kd_arraylen(w, d, false, bad);
                    if (!w.miss) {
                        ver = v;
                        client = cid;
                        if (bad || d.err) done = true;
                        nt = ntp; t = 0;
                        pos = d.pos;
                        st = ST_TOPIC;
                    }
                }
            } else if (kProduce) {
                ReqInfo q;
                q.kind = 0; q.version = ver; q.typed = 1; q.client = client;
                switch (st) {
                case ST_TOPIC: {  // one topic: name (and its rule), partition count
                    if (t >= nt) {  // decoded: MatchesRule over the topics seen
                        done = true;
                        consumed = rawlen;
                        verdict = V_DENY;
                        if (!rs.any) break;
                        const uint32_t best = match_rules(T, rs, q, ntopics, cmax);
                        if (best != kInf) { verdict = V_ALLOW; rule_out = T.rules[rs.rule_first + best].gid; }
                        break;
                    }
                    KD d{pos, rawlen, -1, 0};
                    uint32_t o, l;
                    kd_string(w, d, o, l);
                    if (d.err) { if (!w.miss) done = true; break; }
                    const int32_t tid = l > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, w, o, l) : -1;
                    bool bad = false;
                    const int32_t npp = kd_arraylen(w, d, false, bad);
                    if (w.miss) break;
                    const uint32_t e = topic_first(T, rs, q, tid);
                    ntopics++;
                    cmax = cmax > e ? cmax : e;
                    if (bad || d.err) { done = true; break; }
                    np = npp; p = 0;
                    pos = d.pos;
                    st = ST_PART;
                    break;
                }
                case ST_PART: {  // one partition: id, message-set size
                    if (p >= np) { t++; st = ST_TOPIC; break; }
                    KD d{pos, rawlen, -1, 0};
                    kd_skip(d, 4);
                    if (d.err) { done = true; break; }
                    const int32_t ss = kd_int(w, d, 4);
                    if (w.miss) break;
                    if (d.err) { done = true; break; }
                    pos = d.pos;
                    if (ss < 0) { p++; break; }  // readMessageSet: nothing read
                    if ((uint32_t)ss > kMaxParseBuf) { done = true; break; }
                    slimit = ss;
                    st = ST_MSG;
                    break;
                }
                case ST_MSG: {  // readMessageSet (messages.go:399-492): one message's header
                    KD dec{pos, rawlen, slimit, 0};
                    kd_skip(dec, 8);
                    int32_t msize = 0;
                    bool setend = dec.err != 0;
                    if (!setend) {
                        msize = kd_int(w, dec, 4);
                        setend = dec.err || msize <= 0;
                    }
                    if (w.miss) break;
                    if (!setend && (uint32_t)msize > kMaxParseBuf) { done = true; break; }
                    uint32_t at = 0;
                    if (!setend) {
                        at = kd_read(dec, (uint32_t)msize);
                        setend = dec.err != 0;
                    }
                    if (setend) { pos = dec.pos; slimit = dec.limit; p++; st = ST_PART; break; }
                    KD md{at, at + (uint32_t)msize, -1, 0};
                    const uint32_t sc = (uint32_t)kd_int(w, md, 4);
                    if (msize <= 4) {
                        if (w.miss) break;
                        pos = dec.pos; slimit = dec.limit; p++; st = ST_PART; break;
                    }
                    // the fields after the CRC, decoded now (the window holds the
                    // message's start) and applied once the CRC is known to hold
                    kd_skip(md, 1);
                    const int8_t attr = (int8_t)kd_int(w, md, 1);
                    if (ver >= 1) kd_skip(md, 8);
                    const uint32_t codec = (uint32_t)attr & 3;
                    if (codec != 3) { kd_bytes(w, md); kd_bytes(w, md); }
                    if (w.miss) break;
                    mflags = codec | (md.err ? 4u : 0u);
                    crcst = sc;
                    crc = 0xFFFFFFFFu;
                    crcpos = at + 4;
                    crcend = at + (uint32_t)msize;
                    pos = dec.pos;
                    slimit = dec.limit;
                    st = ST_CRC;
                    break;
                }
                case ST_CRC: {  // CRC32-IEEE of the message body, resident chunks only
                    uint32_t cp = crcpos, c = crc;
                    bool stop = false;
#ifdef KEXP_NOCRC
                    cp = crcend; c = ~crcst;
#endif
                    const uint32_t j0 = (w.a0 + cp) & 15;
                    if (j0 && cp < crcend) {
                        const uint32_t k = (w.a0 + cp) >> 4;
                        if (!w_res(w, k)) stop = true;
                        else {
                            w_fill(w, k);
                            const uint32_t r = 16 - j0 < crcend - cp ? 16 - j0 : crcend - cp;
                            c = crc_in_chunk(tabaddr, w, c, j0, r);
                            cp += r;
                        }
                    }
                    while (!stop && cp + 16 <= crcend) {
                        const uint32_t k = (w.a0 + cp) >> 4;
                        if (!w_res(w, k)) { stop = true; break; }
                        if ((k & 3) == 0 && cp + 64 <= crcend && w_res(w, k + 3)) {
                            const uint32_t la = w.lds + (k & (kWin - 1)) * 1024u;
                            uint4 v0, v1, v2, v3;
                            asm volatile("ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                                         "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\t"
                                         "s_waitcnt lgkmcnt(0)"
                                         : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
                                         : "v"(la)
                                         : "memory");
                            c = crc_step8(tabaddr, v0.x ^ c, v0.y);
                            c = crc_step8(tabaddr, v0.z ^ c, v0.w);
                            c = crc_step8(tabaddr, v1.x ^ c, v1.y);
                            c = crc_step8(tabaddr, v1.z ^ c, v1.w);
                            c = crc_step8(tabaddr, v2.x ^ c, v2.y);
                            c = crc_step8(tabaddr, v2.z ^ c, v2.w);
                            c = crc_step8(tabaddr, v3.x ^ c, v3.y);
                            c = crc_step8(tabaddr, v3.z ^ c, v3.w);
                            cp += 64;
                        } else {
                            const uint4 v = lds_read16(w.lds + (k & (kWin - 1)) * 1024u);
                            c = crc_step8(tabaddr, v.x ^ c, v.y);
                            c = crc_step8(tabaddr, v.z ^ c, v.w);
                            cp += 16;
                        }
                    }
                    if (!stop && cp < crcend) {
                        const uint32_t k = (w.a0 + cp) >> 4;
                        if (!w_res(w, k)) stop = true;
                        else {
                            w_fill(w, k);
                            c = crc_in_chunk(tabaddr, w, c, 0, crcend - cp);
                            cp = crcend;
                        }
                    }
                    crcpos = cp;
                    crc = c;
                    if (stop) { blk = 1; bpos = cp; break; }
                    // the message's effect on the set walk
                    const uint32_t codec = mflags & 3;
                    if (~c != crcst || codec == 3) { p++; st = ST_PART; break; }  // stop, no drain
                    if (mflags & 4) { done = true; break; }
                    if (codec != 0) zflag = 1;
                    st = ST_MSG;
                    break;
                }
                }
            }
            if (w.miss) {
                // a read outside the window: retry from HBM if the window already
                // starts at the step (it is longer than a window), else move it
                if (((w.a0 + spos) >> 4) == w.w0 && !w.gok) {
                    w.gok = 1;
                } else {
                    blk = 1;
                    bpos = spos;
                    w.gok = 0;
                }
                w.miss = 0;
                continue;
            }
            w.gok = 0;
            if (done) {
                if (verdict != V_ALLOW && verdict != V_DENY) consumed = 0;
                B.verdict[idx] = verdict;
                B.rule[idx] = rule_out;
                B.consumed[idx] = consumed;
                if (zflag && zlist && (verdict == V_ALLOW || verdict == V_DENY)) zlist[atomicAdd(zcount, 1u)] = idx;
                st = ST_IDLE;
#ifdef KEXP_STATS
                x_done++;
#endif
            }
        }
    }
#ifdef KEXP_STATS
    {
        const uint32_t d = __builtin_amdgcn_readfirstlane(0) + (uint32_t)__reduce_add_sync(~0ull, x_done);
        uint32_t sst[8];
        for (int k = 0; k < 8; k++) sst[k] = (uint32_t)__reduce_add_sync(~0ull, x_steps[k]);
        if (lane == 0 && (blockIdx.x % 64) == 0 && wave == 0)
            printf("kstats produce=%d block %u rounds %u iters %u done %u active/round %.1f cyc: setup %llu dma %llu proc %llu | steps start %u topic %u part %u msg %u crc %u\n",
                   (int)kProduce, blockIdx.x, x_rounds, x_iters, d, x_rounds ? (double)x_active / x_rounds : 0.0,
                   (unsigned long long)x_tsetup, (unsigned long long)x_tdma, (unsigned long long)x_tproc,
                   sst[ST_START], sst[ST_TOPIC], sst[ST_PART], sst[ST_MSG], sst[ST_CRC]);
    }
#endif
}

hipError_t KafkaPhaseTimes(uint64_t *, bool) { return hipErrorNotSupported; }

// work[0]: the produce kernel's entry counter, work[1]: the other one's (both zeroed by the caller on `stream`)
hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, uint32_t *zlist, uint32_t *zcount, uint32_t *work,
                               hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    if (!sel || !work) return hipErrorInvalidValue;  // the waves walk partition_kernel's lists from the counters
    // persistent grids: as many workgroups as the CUs hold at once
    static int resident[2] = {0, 0};
    for (int k = 0; k < 2; k++) {
        if (resident[k]) continue;
        int dev = 0, cus = 0, per_cu = 0;
        const void *fn = k ? (const void *)kafka_classify_kernel<true> : (const void *)kafka_classify_kernel<false>;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, fn, kBlock, 0) == hipSuccess && cus > 0 && per_cu > 0)
            resident[k] = cus * per_cu;
        else
            resident[k] = 512;
    }
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
    hipLaunchKernelGGL(kafka_classify_kernel<true>, dim3(blocks < (uint32_t)resident[1] ? blocks : resident[1]),
                       dim3(kBlock), 0, stream, B, T, sel, sel_count, answer_other ? 1u : 0u, zlist, zcount, work);
    hipError_t rc = hipGetLastError();
    if (rc != hipSuccess) return rc;
    hipLaunchKernelGGL(kafka_classify_kernel<false>, dim3(blocks < (uint32_t)resident[0] ? blocks : resident[0]),
                       dim3(kBlock), 0, stream, B, T, sel, sel_count, answer_other ? 1u : 0u, zlist, zcount, work + 1);
    return hipGetLastError();
}

}  // namespace l7
