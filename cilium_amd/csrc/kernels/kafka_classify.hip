// Kafka request classification on gfx950 (product code), v2.
//
// One lane per request frame restates, sequentially over its own bytes, the
// reference's decode path: proto.ReadReq framing
// (vendor/github.com/optiopay/kafka/proto/messages.go:124-165), the typed
// decoders (:504-537, :767-824, :1033-1054, :1173-1228, :1389-1430,
// :1591-1647, :1810-1858) with io.ReadFull / LimitReader semantics
// (serialization.go:19-203), readMessageSet (:363-494), then MatchesRule
// (pkg/kafka/policy.go:200-225) against the connection's rule set using the
// precomputed topic / key views (engine/kafka_compile.h).  Compressed message
// sets => L7_UNSUPPORTED.
//
// The message-set CRC32 is where the bytes are (most of a produce request is
// message bodies) and where a one-lane-per-request walk diverges worst: lanes
// hold 0 to dozens of messages of 64 B to KBs.  So every wave works on its 64
// requests in three steps:
//
//   1. speculative walk: each lane decodes its request assuming every message
//      CRC matches; instead of hashing a message body it appends a work item
//      (address, length, stored CRC, lane) to the wave's LDS queue and reads
//      on (magic, attributes, key, value) exactly as the reference does after
//      a matching CRC.  The verdict, rule and consumed length it reaches are
//      the right ones if every queued CRC matches.
//   2. CRC pass: all 64 lanes work off the queue together, one message per
//      lane, 64 bytes per step (four dwordx4 loads, slicing-by-8 with the
//      tables in LDS); a lane that finishes its message takes the next queued
//      one, so the wave stays converged whatever the message sizes.  A
//      mismatch marks the message's lane.
//   3. exact redo: a lane with a mismatching CRC -- or whose queue share ran
//      out -- decodes its request again with the CRC checked inline
//      (readMessageSet stops at a bad CRC without draining the set, so what
//      follows depends on it).  Only adversarial streams get here.
//
// Outputs are written by request index at the end of the tile, so a wave of
// consecutive requests writes whole lines.
#include <hip/hip_runtime.h>

#include "../device_tables.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
constexpr uint32_t kQueue = 192;  // CRC work items per wave (16 B each)
constexpr uint32_t kMaxParseBuf = 6553500;
constexpr uint32_t kInf = 0xFFFFFFFFu;

// ------------------------------------------------------------------ byte cursor
// Each lane keeps the 16-byte aligned chunk it last touched in registers and
// serves field bytes from it (a chunk that holds a request byte never leaves
// the arena's 16-byte rounding; see include/l7gpu.h).
struct Cur {
    uintptr_t line;  // address of the cached chunk (~0 = none)
    uint32_t w[4];
};
__device__ __forceinline__ void cur_fill(Cur &c, uintptr_t a) {
    const uintptr_t ln = a & ~(uintptr_t)15;
    if (ln != c.line) {
        const uint4 v = *reinterpret_cast<const uint4 *>(ln);
        c.w[0] = v.x; c.w[1] = v.y; c.w[2] = v.z; c.w[3] = v.w;
        c.line = ln;
    }
}
__device__ __forceinline__ uint32_t cur_word(const Cur &c, uint32_t k) {
    return k < 8 ? (k < 4 ? c.w[0] : c.w[1]) : (k < 12 ? c.w[2] : c.w[3]);
}
__device__ __forceinline__ uint32_t cur_byte(Cur &c, const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    cur_fill(c, a);
    const uint32_t k = (uint32_t)(a & 15);
    return (cur_word(c, k) >> ((k & 3) * 8)) & 0xFFu;
}
// the 4 bytes at a (little-endian), which lie in one chunk
__device__ __forceinline__ uint32_t cur_le32(Cur &c, uintptr_t a) {
    cur_fill(c, a);
    const uint32_t k = (uint32_t)(a & 15), i = k >> 2;
    const uint32_t lo = i == 0 ? c.w[0] : i == 1 ? c.w[1] : i == 2 ? c.w[2] : c.w[3];
    const uint32_t hi = i == 0 ? c.w[1] : i == 1 ? c.w[2] : c.w[3];
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}
// big-endian n-byte field (n = 1, 2, 4, 8)
__device__ __forceinline__ uint64_t be_load(Cur &c, const uint8_t *p, int n) {
    const uintptr_t a = (uintptr_t)p;
    if (n <= 4 && (a & 15) + 4 <= 16) {
        const uint32_t v = __builtin_bswap32(cur_le32(c, a));
        return n == 4 ? v : v >> (32 - 8 * n);
    }
    if (n == 8 && (a & 15) <= 8) {
        const uint64_t hi = __builtin_bswap32(cur_le32(c, a)), lo = __builtin_bswap32(cur_le32(c, a + 4));
        return hi << 32 | lo;
    }
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | cur_byte(c, p + i);
    return v;
}

// ------------------------------------------------------------------ decoder (serialization.go)
struct KDec {
    const uint8_t *b;
    uint32_t pos, end;
    int64_t limit;  // LimitReader remaining, -1 = none
    int err;        // 0 ok, 1 EOF, 2 ErrUnexpectedEOF, 3 other
    Cur *c;
};

__device__ __forceinline__ uint32_t kavail(const KDec &d) {
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint64_t)d.limit < a) a = (uint32_t)d.limit;
    return a;
}
// io.ReadFull(r, buf[:n]); returns start offset, sets d.err on a short read
__device__ __forceinline__ uint32_t kread(KDec &d, uint32_t n) {
    uint32_t at = d.pos;
    if (n == 0) return at;
    uint32_t a = kavail(d);
    if (a == 0) { d.err = 1; return at; }
    uint32_t take = a < n ? a : n;
    d.pos += take;
    if (d.limit >= 0) d.limit -= take;
    if (take < n) d.err = 2;
    return at;
}
__device__ __forceinline__ int64_t dec_int(KDec &d, int n) {
    if (d.err) return 0;
    uint32_t at = kread(d, (uint32_t)n);
    if (d.err) return 0;
    uint64_t v = be_load(*d.c, d.b + at, n);
    return n == 1 ? (int64_t)(int8_t)v : n == 2 ? (int64_t)(int16_t)v : n == 4 ? (int64_t)(int32_t)v : (int64_t)v;
}
// DecodeString -> (off, len); len < 1 => ""
__device__ __forceinline__ void dec_string(KDec &d, uint32_t &off, uint32_t &len) {
    off = 0; len = 0;
    if (d.err) return;
    int16_t sl = (int16_t)dec_int(d, 2);
    if (d.err || sl < 1) return;
    uint32_t at = kread(d, (uint32_t)sl);
    if (d.err) return;
    off = at; len = (uint32_t)sl;
}
// DecodeArrayLen(nullable): -1 null; sets bad on ErrInvalidArrayLen
__device__ __forceinline__ int64_t dec_arraylen(KDec &d, bool nullable, bool &bad) {
    int64_t l = (int32_t)dec_int(d, 4);
    bad = false;
    if (l < 0) { if (nullable) return -1; bad = true; return 0; }
    if (l > kMaxParseBuf) { bad = true; return 0; }
    return l;
}
__device__ __forceinline__ void dec_bytes(KDec &d) {
    if (d.err) return;
    int32_t sl = (int32_t)dec_int(d, 4);
    if (d.err || sl < 1) return;
    if ((uint32_t)sl > kMaxParseBuf) { d.err = 3; return; }
    kread(d, (uint32_t)sl);
}

// ------------------------------------------------------------------ CRC32-IEEE
// hash/crc32.ChecksumIEEE, slicing-by-8: tab = 8 LDS tables of 256 entries.
__device__ __forceinline__ uint32_t crc_step8(const uint32_t *tab, uint32_t c, uint32_t x, uint32_t y) {
    const uint32_t lo = x ^ c, hi = y;
    return tab[7 * 256 + (lo & 0xFF)] ^ tab[6 * 256 + ((lo >> 8) & 0xFF)] ^ tab[5 * 256 + ((lo >> 16) & 0xFF)] ^
           tab[4 * 256 + (lo >> 24)] ^ tab[3 * 256 + (hi & 0xFF)] ^ tab[2 * 256 + ((hi >> 8) & 0xFF)] ^
           tab[1 * 256 + ((hi >> 16) & 0xFF)] ^ tab[hi >> 24];
}
__device__ __forceinline__ uint32_t crc_byte(const uint32_t *tab, uint32_t c, uint32_t b) {
    return tab[(c ^ b) & 0xFF] ^ (c >> 8);
}
__device__ __forceinline__ uint32_t word_of(const uint4 &v, uint32_t q) {
    return q < 8 ? (q < 4 ? v.x : v.y) : (q < 12 ? v.z : v.w);
}
// one lane, one buffer (exact redo path)
__device__ uint32_t crc32_ieee(const uint32_t *tab, Cur &cur, const uint8_t *p, uint32_t n) {
    uint32_t c = 0xFFFFFFFFu;
    uint32_t i = 0;
    for (; i < n && (((uintptr_t)(p + i)) & 15); i++) c = crc_byte(tab, c, cur_byte(cur, p + i));
    for (; i + 16 <= n; i += 16) {
        const uint4 v = *reinterpret_cast<const uint4 *>(p + i);
        c = crc_step8(tab, c, v.x, v.y);
        c = crc_step8(tab, c, v.z, v.w);
    }
    for (; i < n; i++) c = crc_byte(tab, c, cur_byte(cur, p + i));
    return ~c;
}

// ------------------------------------------------------------------ rule matching
__device__ __forceinline__ int32_t str_lookup(const DevStrSlot *tab, uint32_t mask, const uint8_t *strings, Cur &cur,
                                              const uint8_t *s, uint32_t n) {
    uint32_t h = kFnvBasis;
    for (uint32_t i = 0; i < n; i++) h = (h ^ cur_byte(cur, s + i)) * 16777619u;
    for (uint32_t slot = h & mask;; slot = (slot + 1) & mask) {
        const DevStrSlot e = tab[slot];
        if (!e.used) return -1;
        if (e.hash == h && e.len == n) {
            bool eq = true;
            Cur tc;
            tc.line = ~(uintptr_t)0;
            for (uint32_t i = 0; i < n && eq; i++) eq = cur_byte(tc, strings + e.str_off + i) == cur_byte(cur, s + i);
            if (eq) return e.id;
        }
    }
}

__device__ __forceinline__ bool is_topic_api_key(int k) {
    // 0 1 2 3 4 5 6 8 9 19 20 21 23 24 27 28 34 35 37  (pkg/kafka/policy.go:27-52)
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
__device__ __forceinline__ uint32_t topic_first(const KafkaTables &T, const DevKafkaRuleset &rs, const ReqInfo &q,
                                                int32_t tid) {
    if (tid < 0 || rs.ntopics == 0) return kInf;
    uint32_t off, cnt;
    if (rs.tdense_off != ~0u) {
        const uint2 e = *reinterpret_cast<const uint2 *>(T.index + rs.tdense_off + 2 * (uint32_t)tid);
        off = e.x;
        cnt = e.y;
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

// ------------------------------------------------------------------ per-wave CRC queue
struct Queue {
    uint4 *items;     // {addr lo, addr hi, stored crc, len | lane << 26}
    uint32_t *count;  // items claimed (may exceed kQueue: overflow)
};

// Append a CRC work item for the calling lane; false if the queue is full.
// Called in divergent code: the active lanes take consecutive slots.
__device__ __forceinline__ bool queue_push(const Queue &Q, uint32_t lane, const uint8_t *p, uint32_t n, uint32_t crc) {
    const uint64_t act = __ballot(1);
    const uint32_t leader = (uint32_t)__builtin_ctzll(act);
    const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(act >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)act, 0));
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(Q.count, (uint32_t)__builtin_popcountll(act));
    base = (uint32_t)__shfl((int)base, (int)leader);
    const uint32_t slot = base + rank;
    if (slot >= kQueue || n >= (1u << 26)) return false;
    const uint64_t a = (uint64_t)(uintptr_t)p;
    Q.items[slot] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), crc, n | lane << 26);
    return true;
}

// ------------------------------------------------------------------ one request
enum : int { RS_OK = 0, RS_ERROR = -1, RS_COMPRESSED = -2, RS_OVERFLOW = -3 };

// readMessageSet on the shared position (messages.go:363-494).  kExact: check
// each CRC here; else queue it (assumed to match) and read on.
template <bool kExact>
__device__ __forceinline__ int read_message_set(Cur &cur, const uint8_t *b, uint32_t &pos, uint32_t end, int32_t size,
                                                int16_t version, const uint32_t *crctab, const Queue &Q,
                                                uint32_t lane) {
    if (size < 0) return RS_OK;
    if ((uint32_t)size > kMaxParseBuf) return RS_ERROR;
    KDec dec{b, pos, end, size, 0, &cur};
    int rc = RS_OK;
    for (;;) {
        (void)dec_int(dec, 8);
        if (dec.err) break;
        int32_t msize = (int32_t)dec_int(dec, 4);
        if (dec.err || msize <= 0) break;
        if ((uint32_t)msize > kMaxParseBuf) { rc = RS_ERROR; break; }
        uint32_t at = kread(dec, (uint32_t)msize);
        if (dec.err) break;
        KDec md{b, at, at + (uint32_t)msize, -1, 0, &cur};
        uint32_t crc = (uint32_t)dec_int(md, 4);
        if (msize <= 4) break;
        if (kExact) {
            if (crc != crc32_ieee(crctab, cur, b + at + 4, (uint32_t)msize - 4)) break;  // stop, no drain
        } else if (!queue_push(Q, lane, b + at + 4, (uint32_t)msize - 4, crc)) {
            rc = RS_OVERFLOW;
            break;
        }
        (void)dec_int(md, 1);
        int8_t attr = (int8_t)dec_int(md, 1);
        if (version >= 1) (void)dec_int(md, 8);
        int codec = attr & 3;
        if (codec == 3) break;  // `return nil, err` with err == nil
        dec_bytes(md);
        dec_bytes(md);
        if (md.err) { rc = RS_ERROR; break; }
        if (codec != 0) { rc = RS_COMPRESSED; break; }
    }
    pos = dec.pos;
    return rc;
}

struct Result {
    uint8_t verdict;
    int32_t rule;
    uint32_t consumed;
};

// proto.ReadReq + kafka.ReadRequest + canAccess/MatchesRule for one request.
// Returns false (kExact = false only) if the CRC queue overflowed.
template <bool kExact>
__device__ __forceinline__ bool classify_one(const KafkaTables &T, const DevConn &conn, const uint8_t *b, uint32_t len,
                             const uint32_t *crctab, const Queue &Q, uint32_t lane, Result &out) {
    Cur cur;
    cur.line = ~(uintptr_t)0;
    out.verdict = V_PARSE_ERROR;
    out.rule = -1;
    out.consumed = 0;
    // ---- proto.ReadReq (messages.go:124-165), kafka.ReadRequest (request.go:186-229)
    if (len < 4) { out.verdict = V_INCOMPLETE; return true; }
    const int32_t size = (int32_t)be_load(cur, b, 4);
    if (size <= 0) { out.verdict = V_PARSE_ERROR; return true; }
    if (len < 6) { out.verdict = V_INCOMPLETE; return true; }
    if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) { out.verdict = V_PARSE_ERROR; return true; }
    const uint32_t rawlen = (uint32_t)size + 4;
    if (rawlen > len) { out.verdict = V_INCOMPLETE; return true; }
    if (rawlen < 12) { out.verdict = V_PARSE_ERROR; return true; }
    ReqInfo q;
    q.kind = (int16_t)be_load(cur, b + 4, 2);
    q.version = (int16_t)be_load(cur, b + 6, 2);
    q.typed = (q.kind == 0 || q.kind == 1 || q.kind == 2 || q.kind == 3 || q.kind == 8 || q.kind == 9) ? 1
            : (q.kind == 10 ? 2 : 0);
    q.client = -2;
    const DevKafkaRuleset rs = T.rulesets[conn.ruleset];
    uint32_t ntopics = 0, cmax = 0;  // raw topic count; max over topics of first matching rule
    int rc = RS_OK;
    if (q.typed) {
        KDec d{b, 0, rawlen, -1, 0, &cur};
        bool bad = false;
        (void)dec_int(d, 4); (void)dec_int(d, 2);
        const int16_t ver = (int16_t)dec_int(d, 2);
        (void)dec_int(d, 4);
        uint32_t co, cl;
        dec_string(d, co, cl);
        if (!d.err && cl > 0) q.client = str_lookup(T.client_hash, T.client_mask, T.strings, cur, b + co, cl);
        if (q.client < 0) q.client = -2;
        const bool topics_on = q.typed == 1;
        auto on_topic = [&](uint32_t to, uint32_t tl) {
            if (!topics_on) return;
            ntopics++;
            int32_t tid = tl > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, cur, b + to, tl) : -1;
            uint32_t e = topic_first(T, rs, q, tid);
            cmax = cmax > e ? cmax : e;
        };
        int64_t nt, np;
        uint32_t o, l;
        switch (q.kind) {
        case 0:  // Produce (messages.go:1591-1647)
            if (ver >= 3) dec_string(d, o, l);
            (void)dec_int(d, 2); (void)dec_int(d, 4);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && rc == RS_OK; t++) {
                dec_string(d, o, l);
                if (d.err) break;
                on_topic(o, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = RS_ERROR; break; }
                for (int64_t p = 0; p < np; p++) {
                    (void)dec_int(d, 4);
                    if (d.err) { rc = RS_ERROR; break; }
                    const int32_t ss = (int32_t)dec_int(d, 4);
                    if (d.err) { rc = RS_ERROR; break; }
                    rc = read_message_set<kExact>(cur, b, d.pos, d.end, ss, ver, crctab, Q, lane);
                    if (rc != RS_OK) break;
                }
            }
            break;
        case 1:  // Fetch (messages.go:767-824)
            (void)dec_int(d, 4); (void)dec_int(d, 4); (void)dec_int(d, 4);
            if (ver >= 3) (void)dec_int(d, 4);
            if (ver >= 4) (void)dec_int(d, 1);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o, l);
                on_topic(o, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = RS_ERROR; break; }
                for (int64_t p = 0; p < np && !d.err; p++) {
                    (void)dec_int(d, 4); (void)dec_int(d, 8);
                    if (ver >= 5) (void)dec_int(d, 8);
                    (void)dec_int(d, 4);
                }
            }
            break;
        case 2:  // Offset (messages.go:1810-1858)
            (void)dec_int(d, 4);
            if (ver >= 2) (void)dec_int(d, 1);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o, l);
                on_topic(o, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = RS_ERROR; break; }
                for (int64_t p = 0; p < np && !d.err; p++) {
                    (void)dec_int(d, 4); (void)dec_int(d, 8);
                    if (ver == 0) (void)dec_int(d, 4);
                }
            }
            break;
        case 3:  // Metadata (messages.go:504-537)
            nt = dec_arraylen(d, true, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && !d.err; t++) { dec_string(d, o, l); if (!d.err) on_topic(o, l); }
            if (ver >= 4) (void)dec_int(d, 1);
            break;
        case 8:  // OffsetCommit (messages.go:1173-1228)
            dec_string(d, o, l);
            if (ver >= 1) { (void)dec_int(d, 4); dec_string(d, o, l); }
            if (ver >= 2) (void)dec_int(d, 8);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o, l);
                on_topic(o, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = RS_ERROR; break; }
                for (int64_t p = 0; p < np && !d.err; p++) {
                    (void)dec_int(d, 4); (void)dec_int(d, 8);
                    if (ver == 1) (void)dec_int(d, 8);
                    uint32_t o2, l2;
                    dec_string(d, o2, l2);
                }
            }
            break;
        case 9:  // OffsetFetch (messages.go:1389-1430)
            dec_string(d, o, l);
            nt = dec_arraylen(d, true, bad);
            if (bad) { rc = RS_ERROR; break; }
            for (int64_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o, l);
                on_topic(o, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = RS_ERROR; break; }
                for (int64_t p = 0; p < np && !d.err; p++) (void)dec_int(d, 4);
            }
            break;
        case 10:  // ConsumerMetadata (messages.go:1033-1054)
            dec_string(d, o, l);
            if (ver >= 1) (void)dec_int(d, 1);
            break;
        }
        if (rc == RS_OK && d.err) rc = RS_ERROR;
    }
    if (rc == RS_OVERFLOW) return false;
    if (rc == RS_ERROR) { out.verdict = V_PARSE_ERROR; return true; }
    if (rc == RS_COMPRESSED) { out.verdict = V_UNSUPPORTED; return true; }
    out.consumed = rawlen;
    out.verdict = V_DENY;
    if (!rs.any) return true;  // rules.Kafka == nil => deny (pkg/proxy/kafka.go:139-142)
    // ---- MatchesRule (policy.go:200-225)
    uint32_t best = kInf;
    if (ntopics == 0) {
        const int key = (q.kind >= 0 && q.kind < 64) ? q.kind : 64;
        const uint32_t off = T.index[rs.bykey_off + 2 * key], cnt = T.index[rs.bykey_off + 2 * key + 1];
        for (uint32_t i = 0; i < cnt; i++) {
            uint32_t p = T.index[off + i];
            if (rule_matches(T.rules[rs.rule_first + p], q)) { best = p; break; }
        }
    } else {
        for (uint32_t i = 0; i < rs.ntopicless; i++) {
            uint32_t p = T.index[rs.topicless_off + i];
            if (p >= cmax) break;  // cannot beat topic completion
            if (rule_matches(T.rules[rs.rule_first + p], q)) { best = p; break; }
        }
        if (best == kInf) best = cmax;
    }
    if (best != kInf) { out.verdict = V_ALLOW; out.rule = T.rules[rs.rule_first + best].gid; }
    return true;
}

// The exact decode (CRC checked inline), kept out of line: only lanes with a
// mismatching CRC or an overflowed queue take it.
__device__ __noinline__ void classify_exact(const KafkaTables &T, const DevConn &conn, const uint8_t *b, uint32_t len,
                                            const uint32_t *crctab, Result &out) {
    const Queue none{nullptr, nullptr};
    classify_one<true>(T, conn, b, len, crctab, none, 0, out);
}

// ------------------------------------------------------------------ CRC pass
// All lanes of the wave check the queued message CRCs together.  Lane t
// starts on item t; 64 bytes per step; a lane whose message is done takes the
// next unclaimed item (claims in lane order, by ballot).  Returns the mask of
// request lanes with a mismatching CRC.
struct CrcLane {
    uint64_t a;       // next aligned address
    uint32_t rem;     // bytes left
    uint32_t want;    // stored CRC
    uint32_t owner;   // request lane
    uint32_t c;       // running CRC state
    bool have;
};

__device__ __forceinline__ void crc_load(CrcLane &L, const Queue &Q, uint32_t i, const uint32_t *tab) {
    const uint4 e = Q.items[i];
    L.a = (uint64_t)e.x | (uint64_t)e.y << 32;
    L.want = e.z;
    L.rem = e.w & ((1u << 26) - 1);
    L.owner = e.w >> 26;
    L.c = 0xFFFFFFFFu;
    // bytes up to 16-byte alignment
    const uint32_t k = (uint32_t)(L.a & 15);
    if (k && L.rem) {
        const uint4 v = *reinterpret_cast<const uint4 *>(L.a & ~(uint64_t)15);
        const uint32_t take = min(16u - k, L.rem);
        for (uint32_t j = 0; j < take; j++) {
            const uint32_t q = k + j;
            L.c = crc_byte(tab, L.c, (word_of(v, q) >> ((q & 3) * 8)) & 0xFF);
        }
        L.a += take;
        L.rem -= take;
    }
    L.have = true;
}

__device__ __forceinline__ uint64_t crc_pass(const Queue &Q, uint32_t nitems, const uint32_t *tab, uint32_t lane) {
    uint64_t bad = 0;
    uint32_t next = 64;  // next unclaimed item (wave-uniform)
    CrcLane L;
    L.have = false;
    L.a = 0;
    L.rem = L.want = L.owner = L.c = 0;
    if (lane < nitems) crc_load(L, Q, lane, tab);
    while (__any(L.have)) {
        if (L.have) {
            if (L.rem >= 64) {
                const uint4 *p = reinterpret_cast<const uint4 *>(L.a);
                uint4 v[4];
#pragma unroll
                for (int j = 0; j < 4; j++) v[j] = p[j];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    L.c = crc_step8(tab, L.c, v[j].x, v[j].y);
                    L.c = crc_step8(tab, L.c, v[j].z, v[j].w);
                }
                L.a += 64;
                L.rem -= 64;
            } else {  // tail: < 64 bytes from an aligned address
                for (; L.rem >= 16; L.rem -= 16, L.a += 16) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(L.a);
                    L.c = crc_step8(tab, L.c, v.x, v.y);
                    L.c = crc_step8(tab, L.c, v.z, v.w);
                }
                if (L.rem) {
                    const uint4 v = *reinterpret_cast<const uint4 *>(L.a);
                    for (uint32_t q = 0; q < L.rem; q++) L.c = crc_byte(tab, L.c, (word_of(v, q) >> ((q & 3) * 8)) & 0xFF);
                    L.rem = 0;
                }
                if (~L.c != L.want) bad |= 1ull << L.owner;
                L.have = false;
            }
        }
        // lanes without an item claim the next ones
        const uint64_t idle = __ballot(!L.have);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0));
        if (!L.have && next + rank < nitems) crc_load(L, Q, next + rank, tab);
        next += (uint32_t)__builtin_popcountll(idle);
    }
    // OR the lanes' findings over the wave
    uint32_t lo = (uint32_t)bad, hi = (uint32_t)(bad >> 32);
    for (int o = 32; o > 0; o >>= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o);
        hi |= (uint32_t)__shfl_xor((int)hi, o);
    }
    return (uint64_t)hi << 32 | lo;
}

}  // namespace

// sel: this protocol's request indices (partition_kernel, mixed batches; the
// first sel_count[0] entries), else requests 0..n-1.  answer_other: answer
// entries on connections that are not Kafka (single-protocol engines, where
// partition_kernel does not run).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4, 8))) void kafka_classify_kernel(
    Batch B, KafkaTables T, const uint32_t *__restrict__ sel, const uint32_t *__restrict__ sel_count,
    uint32_t answer_other) {
    __shared__ uint32_t crctab[8 * 256];
    __shared__ uint4 s_items[kWaves][kQueue];
    __shared__ uint32_t s_qn[kWaves];
    __shared__ uint32_t s_verdicts[8];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    {
        uint32_t c = t;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crctab[t] = c;
        if (t < 8) s_verdicts[t] = 0;
        __syncthreads();
        for (int k = 1; k < 8; k++) {
            const uint32_t prev = crctab[(k - 1) * 256 + t];
            crctab[k * 256 + t] = (prev >> 8) ^ crctab[prev & 0xFF];
            __syncthreads();
        }
    }
    const Queue Q{s_items[wave], &s_qn[wave]};
    const uint32_t m = sel ? sel_count[0] : B.n;
    const uint32_t ntiles = (m + 63) / 64;
    uint32_t vcount[5] = {0, 0, 0, 0, 0};
    for (uint32_t tile = blockIdx.x * kWaves + wave; tile < ntiles; tile += gridDim.x * kWaves) {
        const uint32_t i = tile * 64 + lane;
        uint32_t idx = 0;
        bool mine = false, answer = false;
        DevConn conn{-1, PROTO_NONE, 0, {0, 0}};
        uint64_t off = 0;
        uint32_t len = 0;
        Result r{V_UNSUPPORTED, -1, 0};
        if (i < m) {
            idx = sel ? sel[i] : i;
            const uint32_t ci = B.conn_ids[idx];
            if (ci < B.nconns) conn = B.conns[ci];
            mine = conn.proto == PROTO_KAFKA && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets;
            answer = mine || (answer_other && conn.proto != PROTO_HTTP && conn.proto != PROTO_MEMCACHE);
            if (mine) {
                off = B.offs[idx];
                len = B.lens[idx];
                if (!l7_in_arena(off, len, B.arena_len)) mine = false;  // out of contract: UNSUPPORTED
            }
        }
        if (lane == 0) *Q.count = 0;
        __builtin_amdgcn_wave_barrier();
        const uint8_t *b = B.arena + off;
        // 1. speculative walk (CRCs queued)
        bool redo = false;
        if (mine) redo = !classify_one<false>(T, conn, b, len, crctab, Q, lane, r);
        // 2. CRC pass over the queue
        __builtin_amdgcn_wave_barrier();
        const uint32_t nq = min(*(volatile uint32_t *)Q.count, kQueue);
        if (nq) {
            const uint64_t bad = crc_pass(Q, nq, crctab, lane);
            redo |= mine && ((bad >> lane) & 1);
        }
        // 3. exact redo of the lanes a CRC (or the queue) decided against
        if (redo) classify_exact(T, conn, b, len, crctab, r);
        if (answer) {
            B.verdict[idx] = r.verdict;
            B.rule[idx] = r.rule;
            B.consumed[idx] = r.consumed;
            if (B.counters) {
                vcount[r.verdict < 5 ? r.verdict : 4]++;
                if (r.rule >= 0 && (uint32_t)r.rule < B.ncounters - 8)
                    atomicAdd((unsigned long long *)&B.counters[r.rule], 1ull);
            }
        }
        __builtin_amdgcn_wave_barrier();
    }
    if (B.counters) {
        for (int v = 0; v < 5; v++)
            if (vcount[v]) atomicAdd(&s_verdicts[v], vcount[v]);
        __syncthreads();
        if (t < 8 && s_verdicts[t])
            atomicAdd((unsigned long long *)&B.counters[B.ncounters - 8 + t], (unsigned long long)s_verdicts[t]);
    }
}

hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    const uint32_t ntiles = (B.n + 63) / 64;
    uint32_t blocks = (ntiles + kWaves - 1) / kWaves;
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(kafka_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                       answer_other ? 1u : 0u);
    return hipGetLastError();
}

}  // namespace l7
