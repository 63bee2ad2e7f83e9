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

// Optional per-phase cycle accounting (-DL7G_KX_TIMING, experiment builds):
// 0 framing, 1 walk loop, 2 CRC pass, 3 topic lookups, 4 verdict + output,
// 5 walk iterations, 6 window refills, 7 tiles.
#ifdef L7G_KX_TIMING
__device__ unsigned long long g_kx_phase[8];
#define KX_DECL uint64_t kx_t = __builtin_amdgcn_s_memtime(); uint64_t kx_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#define KX_MARK(slot) do { const uint64_t kx_n = __builtin_amdgcn_s_memtime(); kx_acc[slot] += kx_n - kx_t; kx_t = kx_n; } while (0)
#define KX_COUNT(slot, v) (kx_acc[slot] += (v))
#define KX_FLUSH(lane) do { if ((lane) == 0) for (int kx_i = 0; kx_i < 8; kx_i++) atomicAdd(&g_kx_phase[kx_i], (unsigned long long)kx_acc[kx_i]); } while (0)
#else
#define KX_DECL
#define KX_MARK(slot) do {} while (0)
#define KX_COUNT(slot, v) do {} while (0)
#define KX_FLUSH(lane) do {} while (0)
#endif
constexpr uint32_t kQueue = 192;  // CRC work items per wave (16 B each)
constexpr uint32_t kMaxParseBuf = 6553500;
constexpr uint32_t kInf = 0xFFFFFFFFu;

// ------------------------------------------------------------------ byte cursor
// Each lane keeps the 16-byte aligned chunk it last touched in registers and
// serves field bytes from it (a chunk that holds a request byte never leaves
// the arena's 16-byte rounding; see include/l7gpu.h).
struct Cur {
    uintptr_t line;  // address of the cached chunk (~0 = none)
    uint32_t w0, w1, w2, w3;  // scalars, not an array: a selected array element would put Cur in scratch
};
__device__ __forceinline__ void cur_fill(Cur &c, uintptr_t a) {
    const uintptr_t ln = a & ~(uintptr_t)15;
    if (ln != c.line) {
        const uint4 v = *reinterpret_cast<const uint4 *>(ln);
        c.w0 = v.x; c.w1 = v.y; c.w2 = v.z; c.w3 = v.w;
        c.line = ln;
    }
}
// (values are copied out before they are selected: a select between struct
// members becomes a select between their addresses, i.e. a scratch array)
__device__ __forceinline__ uint32_t cur_word(const Cur &c, uint32_t k) {
    const uint32_t a = c.w0, b = c.w1, d = c.w2, e = c.w3;
    return k < 8 ? (k < 4 ? a : b) : (k < 12 ? d : e);
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
    const uint32_t w0 = c.w0, w1 = c.w1, w2 = c.w2, w3 = c.w3;
    const uint32_t lo = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
    const uint32_t hi = i == 0 ? w1 : i == 1 ? w2 : w3;
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
    const uint32_t x = v.x, y = v.y, z = v.z, w = v.w;  // values, not member addresses (see cur_word)
    return q < 8 ? (q < 4 ? x : y) : (q < 12 ? z : w);
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

// ------------------------------------------------------------------ exact decode (redo path)
// The reference's decode of one request, sequential, CRC checked inline.
// Lanes whose request the fast path cannot finish exactly (a message CRC that
// does not match) take it; it is kept out of line.
enum : int { RS_OK = 0, RS_ERROR = -1, RS_COMPRESSED = -2 };

// readMessageSet on the shared position (messages.go:363-494)
__device__ __forceinline__ int read_message_set(Cur &cur, const uint8_t *b, uint32_t &pos, uint32_t end, int32_t size,
                                                int16_t version, const uint32_t *crctab) {
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
        if (crc != crc32_ieee(crctab, cur, b + at + 4, (uint32_t)msize - 4)) break;  // stop, no drain
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

// MatchesRule (policy.go:200-225) from the raw topic count and the topic
// completion index cmax (max over topics of the first rule that matches it)
__device__ __forceinline__ void match_rules(const KafkaTables &T, const DevKafkaRuleset &rs, const ReqInfo &q,
                                            uint32_t ntopics, uint32_t cmax, uint32_t rawlen, Result &out) {
    out.consumed = rawlen;
    out.verdict = V_DENY;
    out.rule = -1;
    if (!rs.any) return;  // rules.Kafka == nil => deny (pkg/proxy/kafka.go:139-142)
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
}

// proto.ReadReq framing checks; false = answered (out set), else rawlen / kind / version
__device__ __forceinline__ bool frame_request(Cur &cur, const uint8_t *b, uint32_t len, Result &out, uint32_t &rawlen,
                                              ReqInfo &q) {
    out.verdict = V_PARSE_ERROR;
    out.rule = -1;
    out.consumed = 0;
    // proto.ReadReq (messages.go:124-165), kafka.ReadRequest (request.go:186-229)
    if (len < 4) { out.verdict = V_INCOMPLETE; return false; }
    const int32_t size = (int32_t)be_load(cur, b, 4);
    if (size <= 0) { out.verdict = V_PARSE_ERROR; return false; }
    if (len < 6) { out.verdict = V_INCOMPLETE; return false; }
    if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) { out.verdict = V_PARSE_ERROR; return false; }
    rawlen = (uint32_t)size + 4;
    if (rawlen > len) { out.verdict = V_INCOMPLETE; return false; }
    if (rawlen < 12) { out.verdict = V_PARSE_ERROR; return false; }
    q.kind = (int16_t)be_load(cur, b + 4, 2);
    q.version = (int16_t)be_load(cur, b + 6, 2);
    q.typed = (q.kind == 0 || q.kind == 1 || q.kind == 2 || q.kind == 3 || q.kind == 8 || q.kind == 9) ? 1
            : (q.kind == 10 ? 2 : 0);
    q.client = -2;
    return true;
}

__device__ __forceinline__ void classify_exact(const KafkaTables &T, const DevConn &conn, const uint8_t *b, uint32_t len,
                                            const uint32_t *crctab, Result &out) {
    Cur cur;
    cur.line = ~(uintptr_t)0;
    uint32_t rawlen = 0;
    ReqInfo q;
    if (!frame_request(cur, b, len, out, rawlen, q)) return;
    const DevKafkaRuleset rs = T.rulesets[conn.ruleset];
    uint32_t ntopics = 0, cmax = 0;
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
                    rc = read_message_set(cur, b, d.pos, d.end, ss, ver, crctab);
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
    if (rc == RS_ERROR) { out.verdict = V_PARSE_ERROR; out.consumed = 0; return; }
    if (rc == RS_COMPRESSED) { out.verdict = V_UNSUPPORTED; out.consumed = 0; return; }
    match_rules(T, rs, q, ntopics, cmax, rawlen, out);
}

// ------------------------------------------------------------------ fast path: the decode as a program
// The typed decoders are sequences of the same few field operations, so each
// kind is a small program (kProg) that every lane interprets over its own
// bytes.  A lane only touches memory for the integer fields it must look at
// (array lengths, sizes, message headers): those come from a 32-byte window
// of its request held in registers.  When a lane's next field lies outside its
// window, the lane stops; the wave then refills every stopped lane's window
// together (one pair of dwordx4 loads, all latencies overlapped) and the lanes
// run on.  Strings and fixed-size fields nobody looks at are skipped by length
// alone.  Two things are queued per wave instead of done in the walk:
//   * message CRCs (checked by the wave together, see crc_pass);
//   * topic names (looked up by the wave together, one topic per lane,
//     see flush_topics) -- MatchesRule needs only the topic count and the max
//     over topics of the first rule that matches each (cmax).
enum : uint8_t {
    P_END = 0,   // program done
    P_SKIP,      // a: bytes of fixed-size ints read and dropped
    P_SKIP_VGE,  // the same if version >= b
    P_SKIP_VEQ,  // the same if version == b
    P_STR,       // DecodeString, dropped
    P_STR_VGE,   // the same if version >= b
    P_CLIENT,    // DecodeString: the client id
    P_TOPIC,     // DecodeString: a topic (GetTopics entry), counted even on error
    P_TOPIC_OK,  // DecodeString: a topic, counted only without error
    P_ARR,       // DecodeArrayLen (a: nullable), b: loop level; skips to after the matching P_NEXT if empty
    P_NEXT,      // end of a loop body (b: level): next element (no decoder error) or fall through
    P_PART,      // produce partition: id, set size, readMessageSet
    P_ARRSK,     // DecodeArrayLen of fixed-size elements nobody looks at: the loop is one skip of
                 // count * (a + extra) bytes (b: extra = 1: 8 if version >= 5, 2: 4 if version == 0)
};
struct POp {
    uint8_t op, a, b, jump;  // jump: P_ARR -> index after its P_NEXT; P_NEXT -> body start
};
#define PO(o, a, b, j) {o, a, b, j}
// kinds 0, 1, 2, 3, 8, 9, 10 at these offsets (messages.go decoders, see classify_exact)
__constant__ POp kProg[] = {
    // 0: Produce (:1591-1647)
    PO(P_CLIENT, 0, 0, 0), PO(P_STR_VGE, 0, 3, 0), PO(P_SKIP, 6, 0, 0), PO(P_ARR, 0, 0, 9),
    PO(P_TOPIC_OK, 0, 0, 0), PO(P_ARR, 0, 1, 8), PO(P_PART, 0, 0, 0), PO(P_NEXT, 0, 1, 6), PO(P_NEXT, 0, 0, 4),
    PO(P_END, 0, 0, 0),
    // 10: Fetch (:767-824)
    PO(P_CLIENT, 0, 0, 0), PO(P_SKIP, 12, 0, 0), PO(P_SKIP_VGE, 4, 3, 0), PO(P_SKIP_VGE, 1, 4, 0),
    PO(P_ARR, 0, 0, 18), PO(P_TOPIC, 0, 0, 0), PO(P_ARRSK, 16, 1, 0), PO(P_NEXT, 0, 0, 15), PO(P_END, 0, 0, 0),
    // 19: Offset (:1810-1858)
    PO(P_CLIENT, 0, 0, 0), PO(P_SKIP, 4, 0, 0), PO(P_SKIP_VGE, 1, 2, 0), PO(P_ARR, 0, 0, 26), PO(P_TOPIC, 0, 0, 0),
    PO(P_ARRSK, 12, 2, 0), PO(P_NEXT, 0, 0, 23), PO(P_END, 0, 0, 0),
    // 27: Metadata (:504-537)
    PO(P_CLIENT, 0, 0, 0), PO(P_ARR, 1, 0, 31), PO(P_TOPIC_OK, 0, 0, 0), PO(P_NEXT, 0, 0, 29),
    PO(P_SKIP_VGE, 1, 4, 0), PO(P_END, 0, 0, 0),
    // 33: OffsetCommit (:1173-1228)
    PO(P_CLIENT, 0, 0, 0), PO(P_STR, 0, 0, 0), PO(P_SKIP_VGE, 4, 1, 0), PO(P_STR_VGE, 0, 1, 0),
    PO(P_SKIP_VGE, 8, 2, 0), PO(P_ARR, 0, 0, 46), PO(P_TOPIC, 0, 0, 0), PO(P_ARR, 0, 1, 45), PO(P_SKIP, 12, 0, 0),
    PO(P_SKIP_VEQ, 8, 1, 0), PO(P_STR, 0, 0, 0), PO(P_NEXT, 0, 1, 41), PO(P_NEXT, 0, 0, 39), PO(P_END, 0, 0, 0),
    // 47: OffsetFetch (:1389-1430)
    PO(P_CLIENT, 0, 0, 0), PO(P_STR, 0, 0, 0), PO(P_ARR, 1, 0, 53), PO(P_TOPIC, 0, 0, 0), PO(P_ARRSK, 4, 0, 0),
    PO(P_NEXT, 0, 0, 50), PO(P_END, 0, 0, 0),
    // 54: ConsumerMetadata (:1033-1054)
    PO(P_CLIENT, 0, 0, 0), PO(P_STR, 0, 0, 0), PO(P_SKIP_VGE, 1, 1, 0), PO(P_END, 0, 0, 0),
};
#undef PO
constexpr uint32_t kProgLen = 58;
static_assert(sizeof(kProg) == kProgLen * sizeof(POp), "program table");
static_assert(kProgLen <= kBlock, "one thread per program entry");
__device__ __forceinline__ uint32_t prog_start(int kind) {
    return kind == 0 ? 0 : kind == 1 ? 10 : kind == 2 ? 19 : kind == 3 ? 27 : kind == 8 ? 33 : kind == 9 ? 47 : 54;
}

// message-set sub-states (readMessageSet, messages.go:363-494)
enum : uint8_t { M_NONE = 0, M_HEAD, M_CRC, M_KEY, M_VALUE };

// 32-byte register window of a lane's request, as four 64-bit words
struct Win {
    uint64_t wa;  // address of q0's first byte (16-byte aligned)
    uint64_t q0, q1, q2, q3;  // scalars: an indexed array would live in scratch
};
__device__ __forceinline__ bool win_has(const Win &W, uint64_t a, uint32_t n) { return a >= W.wa && a + n <= W.wa + 32; }
// big-endian value of the vn (1..8) bytes at a; win_has(W, a, vn)
__device__ __forceinline__ uint64_t win_be(const Win &W, uint64_t a, uint32_t vn) {
    const uint32_t k = (uint32_t)(a - W.wa), i = k >> 3, sh = (k & 7) * 8;
    const uint64_t x0 = W.q0, x1 = W.q1, x2 = W.q2, x3 = W.q3;
    const uint64_t lo = i == 0 ? x0 : i == 1 ? x1 : i == 2 ? x2 : x3;
    const uint64_t hi = i == 0 ? x1 : i == 1 ? x2 : x3;
    const uint64_t le = sh ? (lo >> sh) | (hi << (64 - sh)) : lo;  // the 8 bytes at a, little-endian
    const uint64_t be = (uint64_t)__builtin_bswap32((uint32_t)le) << 32 | __builtin_bswap32((uint32_t)(le >> 32));
    return be >> (64 - 8 * vn);
}

struct Walk {
    // outer decoder (bytes.Buffer over rawMsg) and readMessageSet's LimitReader
    // decoder share pos; the message decoder has its own (mpos)
    uint32_t pos, end, mpos, mend, slim;
    bool err, serr, merr;  // sticky decoder errors
    // program
    uint32_t pc;
    int32_t cnt0, cnt1;  // remaining elements of the topic / partition loop
    int rc;              // RS_OK / RS_ERROR / RS_COMPRESSED
    bool done;
    uint32_t ms;         // M_* sub-state (readMessageSet)
    uint32_t at;         // current message body start
    int codec;
    // findings
    uint32_t ntopics;
    uint32_t client_off, client_len;
    // window request
    bool need;
    uint32_t need_pos;   // request position the window must cover
    // queued work (pushed by the wave at the end of the round)
    bool has_crc, has_topic;
    uint32_t crc_off, crc_len, crc_want, top_off, top_len;
};

// io.ReadFull of n bytes that nobody looks at: bounds only (sticky error E,
// a short read advances P to the bound)
__device__ __forceinline__ bool rd_skip(uint32_t &P, uint32_t lim, bool &E, uint32_t n) {
    if (E || n == 0) return !E;
    const uint32_t avail = lim > P ? lim - P : 0;
    if (avail == 0) { E = true; return false; }
    if (avail < n) { P += avail; E = true; return false; }
    P += n;
    return true;
}

// One step of a lane's walk: one field (or a fixed group of fields with the
// same error outcome) read through one common path.  false = stop (window
// needed, an item pending already, or done).
__device__ __forceinline__ bool walk_step(Walk &S, const Win &W, const uint8_t *b, int ver, const POp *prog) {
    // ---- A. what the step reads: n bytes on decoder dec (0 outer, 1 set, 2 message),
    //         the value is the last vn of them
    POp o{0, 0, 0, 0};
    uint32_t dec = 0, n = 0, vn = 0;
    const uint32_t ms = S.ms;
    if (ms != M_NONE) {
        // readMessageSet (messages.go:363-494): offset i64 + size i32 (one
        // outcome: any short read ends the set), crc u32, magic + attributes,
        // timestamp i64 (version >= 1), key / value i32 lengths
        dec = ms == M_HEAD ? 1 : 2;
        // M_CRC: crc u32 + magic i8 + attributes i8 (the body holds >= 5 bytes;
        // a missing attributes byte is a short read of the message decoder)
        n = ms == M_HEAD ? 12 : ms == M_CRC ? min(6u, S.mend - S.mpos) : 4;
        vn = ms == M_HEAD ? 4 : n;
    } else {
        o = prog[S.pc];
        if (o.op == P_STR || o.op == P_STR_VGE || o.op == P_CLIENT || o.op == P_TOPIC || o.op == P_TOPIC_OK) {
            if (o.op != P_STR_VGE || ver >= o.b) n = vn = 2;  // DecodeString: i16 length
        } else if (o.op == P_ARR || o.op == P_ARRSK) {
            n = vn = 4;  // DecodeArrayLen: i32
        } else if (o.op == P_PART) {
            n = 8;  // partition id i32 + set size i32 (either short read is fatal)
            vn = 4;
        }
    }
    // ---- B. the read (io.ReadFull semantics: nothing left => EOF, a partial
    //         read advances the position; errors are sticky)
    uint32_t P = dec == 2 ? S.mpos : S.pos;
    const uint32_t lim = dec == 0 ? S.end : dec == 1 ? min(S.end, S.slim) : S.mend;
    bool E = dec == 0 ? S.err : dec == 1 ? S.serr : S.merr;
    uint64_t v = 0;
    bool ok = true;  // value read
    if (n) {
        if (E) {
            ok = false;
        } else {
            const uint32_t avail = lim > P ? lim - P : 0;
            if (avail < n) {
                P += avail;
                E = true;
                ok = false;
            } else {
                const uint64_t a = (uint64_t)(uintptr_t)(b + P);
                if (!win_has(W, a, n)) {
                    S.need = true;
                    S.need_pos = P;
                    return false;
                }
                v = win_be(W, a + n - vn, vn);
                P += n;
            }
        }
        if (dec == 2) { S.mpos = P; S.merr = E; }
        else if (dec == 1) { S.pos = P; S.serr = E; }
        else { S.pos = P; S.err = E; }
    }
    // ---- C. what the value means
    if (ms != M_NONE) {
        if (ms == M_HEAD) {
            const int32_t msize = (int32_t)(uint32_t)v;
            if (!ok || msize <= 0) { S.ms = M_NONE; return true; }  // the set ends
            if ((uint32_t)msize > kMaxParseBuf) { S.rc = RS_ERROR; S.done = true; return false; }
            const uint32_t at = S.pos;
            if (!rd_skip(S.pos, min(S.end, S.slim), S.serr, (uint32_t)msize)) { S.ms = M_NONE; return true; }
            if (msize <= 4) { S.ms = M_NONE; return true; }  // crc only: appended, the set stops
            S.at = at;
            S.mend = at + (uint32_t)msize;
            S.mpos = at;
            S.merr = false;
            S.ms = M_CRC;
            return true;
        }
        if (ms == M_CRC) {  // the body holds > 4 bytes: the crc is there; queue the check
            if (S.has_crc) { S.mpos -= n; return false; }  // one item per lane per round
            S.has_crc = true;
            S.crc_off = S.at + 4;
            S.crc_len = S.mend - S.at - 4;
            S.crc_want = (uint32_t)(v >> (8 * (n - 4)));
            if (n < 6) S.merr = true;  // attributes missing: short read (codec 0)
            S.codec = n == 6 ? (int)(v & 3) : 0;
            if (ver >= 1) rd_skip(S.mpos, S.mend, S.merr, 8);  // timestamp i64
            S.ms = S.codec == 3 ? M_NONE : M_KEY;  // codec 3: `return nil, nil`
            return true;
        }
        // M_KEY / M_VALUE: DecodeBytes (< 1 => nil, > max => error, else the bytes)
        if (ok) {
            const int32_t sl = (int32_t)(uint32_t)v;
            if (sl >= 1) {
                if ((uint32_t)sl > kMaxParseBuf) S.merr = true;
                else rd_skip(S.mpos, S.mend, S.merr, (uint32_t)sl);
            }
        }
        if (ms == M_KEY) { S.ms = M_VALUE; return true; }
        if (S.merr) { S.rc = RS_ERROR; S.done = true; return false; }
        if (S.codec != 0) { S.rc = RS_COMPRESSED; S.done = true; return false; }
        S.ms = M_HEAD;  // next message
        return true;
    }
    switch (o.op) {
    case P_END:
        S.done = true;
        return false;
    case P_SKIP_VGE:
    case P_SKIP_VEQ:
    case P_SKIP:
        if (o.op == P_SKIP || (o.op == P_SKIP_VGE ? ver >= o.b : ver == o.b)) rd_skip(S.pos, S.end, S.err, o.a);
        S.pc++;
        return true;
    case P_ARR: {
        int32_t l = (int32_t)(uint32_t)v;  // 0 after an error
        if (l < 0) {
            if (!o.a) { S.rc = RS_ERROR; S.done = true; return false; }  // ErrInvalidArrayLen
            l = 0;  // null array
        }
        if ((uint32_t)l > kMaxParseBuf) { S.rc = RS_ERROR; S.done = true; return false; }
        if (o.b == 0) S.cnt0 = l; else S.cnt1 = l;
        S.pc = (l > 0 && !S.err) ? S.pc + 1 : o.jump;
        return true;
    }
    case P_ARRSK: {
        const int32_t l = (int32_t)(uint32_t)v;  // 0 after an error
        if (l < 0 || (uint32_t)l > kMaxParseBuf) { S.rc = RS_ERROR; S.done = true; return false; }
        const uint32_t sz = o.a + (o.b == 1 ? (ver >= 5 ? 8u : 0u) : o.b == 2 ? (ver == 0 ? 4u : 0u) : 0u);
        if (l > 0) rd_skip(S.pos, S.end, S.err, (uint32_t)l * sz);  // <= 6,553,500 * 24: no overflow
        S.pc++;
        return true;
    }
    case P_NEXT: {
        const int32_t c = (o.b == 0 ? S.cnt0 : S.cnt1) - 1;
        if (o.b == 0) S.cnt0 = c; else S.cnt1 = c;
        S.pc = (c > 0 && !S.err) ? o.jump : S.pc + 1;
        return true;
    }
    case P_PART: {
        if (!ok) { S.rc = RS_ERROR; S.done = true; return false; }
        const int32_t ss = (int32_t)(uint32_t)v;
        S.pc++;
        if (ss < 0) return true;  // null set
        if ((uint32_t)ss > kMaxParseBuf) { S.rc = RS_ERROR; S.done = true; return false; }
        S.slim = S.pos + (uint32_t)ss;
        S.serr = false;
        S.ms = M_HEAD;
        return true;
    }
    default: {  // strings: P_STR, P_STR_VGE, P_CLIENT, P_TOPIC, P_TOPIC_OK
        if (o.op == P_STR_VGE && ver < o.b) { S.pc++; return true; }
        const bool topic = o.op == P_TOPIC || o.op == P_TOPIC_OK;
        if (topic && S.has_topic) {  // one topic per lane per round: this step again next round
            if (ok) S.pos -= 2;  // (after a failed read the sticky error makes the redo identical)
            return false;
        }
        const int32_t sl = (int16_t)(uint16_t)v;
        uint32_t so = 0, sn = 0;
        if (ok && sl >= 1) {
            const uint32_t at = S.pos;
            if (rd_skip(S.pos, S.end, S.err, (uint32_t)sl)) { so = at; sn = (uint32_t)sl; }
        }
        S.pc++;
        if (o.op == P_CLIENT) {
            if (!S.err) { S.client_off = so; S.client_len = sn; }
        } else if (o.op == P_TOPIC || (o.op == P_TOPIC_OK && !S.err)) {
            S.has_topic = true;
            S.top_off = so;
            S.top_len = sn;
            S.ntopics++;
        }
        return true;
    }
    }
}

// ------------------------------------------------------------------ per-wave queues
struct WaveLds {
    // CRC work items: request offset, length | lane << 26, stored CRC
    uint32_t *c_off, *c_len, *c_want;
    // topic names: request offset, length | lane << 26
    uint32_t *t_off, *t_len;
    // per request lane
    const uint8_t **base;  // request start
    uint32_t *cmax;        // max over its topics of the first matching rule (atomicMax)
    int32_t *rs;           // rule set
    int32_t *client;       // interned client id (-2 none)
    int32_t *kind, *ver;
};
constexpr uint32_t kCrcQ = 320;   // CRC items per wave (cfg3: ~160 per 64 requests)
constexpr uint32_t kTopQ = 320;   // topics per wave (cfg3: ~140 per 64 requests)

// CRC pass over items [0, n): lane t starts on item t, 64 bytes per step; a
// lane whose message is done takes the next unclaimed item.  ORs the request
// lanes with a mismatching CRC into bad.
struct CrcLane {
    uint64_t a;       // next address
    uint32_t rem;     // bytes left
    uint32_t want;    // stored CRC
    uint32_t owner;   // request lane
    uint32_t c;       // running CRC state
    bool have;
};
__device__ __forceinline__ void crc_load(CrcLane &L, const WaveLds &Q, uint32_t i, const uint32_t *tab) {
    L.owner = Q.c_len[i] >> 26;
    L.rem = Q.c_len[i] & ((1u << 26) - 1);
    L.want = Q.c_want[i];
    L.a = (uint64_t)(uintptr_t)Q.base[L.owner] + Q.c_off[i];
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
__device__ __forceinline__ uint64_t crc_pass(const WaveLds &Q, uint32_t nitems, const uint32_t *tab, uint32_t lane) {
    uint64_t bad = 0;
    uint32_t next = 64;  // next unclaimed item (wave-uniform)
    CrcLane L;
    L.have = false;
    L.a = 0;
    L.rem = L.want = L.owner = L.c = 0;
    if (lane < nitems) crc_load(L, Q, lane, tab);
    // 64-byte blocks are software-pipelined: the next block of the lane's
    // message is loaded while the current one is hashed
    uint4 pf0 = make_uint4(0, 0, 0, 0), pf1 = pf0, pf2 = pf0, pf3 = pf0;
    bool haspf = false;
    while (__any(L.have)) {
        if (L.have) {
            if (L.rem >= 64) {
                uint4 v0, v1, v2, v3;
                if (haspf) {
                    v0 = pf0; v1 = pf1; v2 = pf2; v3 = pf3;
                } else {
                    const uint4 *p = reinterpret_cast<const uint4 *>(L.a);
                    v0 = p[0]; v1 = p[1]; v2 = p[2]; v3 = p[3];
                }
                haspf = L.rem >= 128;  // the next block lies inside the message
                if (haspf) {
                    const uint4 *q = reinterpret_cast<const uint4 *>(L.a + 64);
                    pf0 = q[0]; pf1 = q[1]; pf2 = q[2]; pf3 = q[3];
                }
                L.c = crc_step8(tab, L.c, v0.x, v0.y);
                L.c = crc_step8(tab, L.c, v0.z, v0.w);
                L.c = crc_step8(tab, L.c, v1.x, v1.y);
                L.c = crc_step8(tab, L.c, v1.z, v1.w);
                L.c = crc_step8(tab, L.c, v2.x, v2.y);
                L.c = crc_step8(tab, L.c, v2.z, v2.w);
                L.c = crc_step8(tab, L.c, v3.x, v3.y);
                L.c = crc_step8(tab, L.c, v3.z, v3.w);
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
        const uint64_t idle = __ballot(!L.have);
        const uint32_t rank = __builtin_amdgcn_mbcnt_hi((uint32_t)(idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)idle, 0));
        if (!L.have && next + rank < nitems) {
            crc_load(L, Q, next + rank, tab);
            haspf = false;
        }
        next += (uint32_t)__builtin_popcountll(idle);
    }
    uint32_t lo = (uint32_t)bad, hi = (uint32_t)(bad >> 32);
    for (int o = 32; o > 0; o >>= 1) {
        lo |= (uint32_t)__shfl_xor((int)lo, o);
        hi |= (uint32_t)__shfl_xor((int)hi, o);
    }
    return (uint64_t)hi << 32 | lo;
}

// Topic lookups for queued names [0, n): one name per lane.  Each name's
// first matching rule position (kInf: none) is max-ed into its request lane.
__device__ __forceinline__ void flush_topics(const KafkaTables &T, const WaveLds &Q, uint32_t n, uint32_t lane) {
    for (uint32_t i = lane; i < n; i += 64) {
        const uint32_t owner = Q.t_len[i] >> 26, tl = Q.t_len[i] & ((1u << 26) - 1);
        const uint8_t *b = Q.base[owner];
        ReqInfo q;
        q.kind = Q.kind[owner];
        q.version = Q.ver[owner];
        q.typed = 1;
        q.client = Q.client[owner];
        Cur cur;
        cur.line = ~(uintptr_t)0;
        const int32_t tid = tl > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, cur, b + Q.t_off[i], tl) : -1;
        const DevKafkaRuleset rs = T.rulesets[Q.rs[owner]];
        const uint32_t e = topic_first(T, rs, q, tid);
        atomicMax(&Q.cmax[owner], e);
    }
}

}  // namespace

// sel: this protocol's request indices (partition_kernel, mixed batches; the
// first sel_count[0] entries), else requests 0..n-1.  answer_other: answer
// entries on connections that are not Kafka (single-protocol engines, where
// partition_kernel does not run).
__global__ __launch_bounds__(kBlock) void kafka_classify_kernel(Batch B, KafkaTables T,
                                                                const uint32_t *__restrict__ sel,
                                                                const uint32_t *__restrict__ sel_count,
                                                                uint32_t answer_other) {
    __shared__ uint32_t crctab[8 * 256];
    __shared__ uint32_t s_c[kWaves][3][kCrcQ];
    __shared__ uint32_t s_t[kWaves][2][kTopQ];
    __shared__ const uint8_t *s_base[kWaves][64];
    __shared__ uint32_t s_cmax[kWaves][64];
    __shared__ int32_t s_req[kWaves][4][64];
    __shared__ uint32_t s_verdicts[8];
    __shared__ POp s_prog[kProgLen];
    const uint32_t t = threadIdx.x, lane = t & 63, wave = t >> 6;
    if (t < kProgLen) s_prog[t] = kProg[t];
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
    const WaveLds Q{s_c[wave][0], s_c[wave][1], s_c[wave][2], s_t[wave][0], s_t[wave][1], s_base[wave],
                    s_cmax[wave], s_req[wave][0], s_req[wave][1], s_req[wave][2], s_req[wave][3]};
    const uint32_t m = sel ? sel_count[0] : B.n;
    const uint32_t ntiles = (m + 63) / 64;
    uint32_t vcount[5] = {0, 0, 0, 0, 0};
    KX_DECL
    for (uint32_t tile = blockIdx.x * kWaves + wave; tile < ntiles; tile += gridDim.x * kWaves) {
        KX_COUNT(7, 1);
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
        const uint8_t *b = B.arena + off;
        // ---- framing (ReadReq) and the request header
        uint32_t rawlen = 0;
        ReqInfo q{0, 0, 0, -2};
        bool walk = false;
        if (mine) {
            Cur cur;
            cur.line = ~(uintptr_t)0;
            walk = frame_request(cur, b, len, r, rawlen, q);
        }
        Walk S;
        S.pos = 12;
        S.end = rawlen;
        S.err = false;
        S.pc = prog_start(q.kind);
        S.cnt0 = S.cnt1 = 0;
        S.rc = RS_OK;
        S.done = !walk || !q.typed;  // untyped kinds: request = nil, nothing to decode
        S.ms = M_NONE;
        S.serr = S.merr = false;
        S.slim = 0;
        S.at = S.mend = S.mpos = 0;
        S.codec = 0;
        S.ntopics = 0;
        S.client_off = S.client_len = 0;
        S.need = !S.done;
        S.need_pos = 12;
        S.has_crc = S.has_topic = false;
        Win W;
        W.wa = ~0ull;
        Q.base[lane] = b;
        Q.cmax[lane] = 0;
        Q.rs[lane] = conn.ruleset;
        Q.kind[lane] = q.kind;
        Q.ver[lane] = q.version;
        uint32_t nc = 0, nt = 0;  // queued CRC items / topics (wave-uniform)
        bool ovf = false;         // a queue was full: exact redo
        bool client_done = false;
        const uint64_t req_end = (uint64_t)(uintptr_t)b + len;
        KX_MARK(0);
        while (__any(!S.done)) {
            KX_COUNT(5, 1);
            KX_COUNT(6, __builtin_popcountll(__ballot(!S.done && S.need)));
            // refill the windows of the lanes that stopped on one (all loads in flight together)
            if (!S.done && S.need) {
                W.wa = (uint64_t)(uintptr_t)(b + S.need_pos) & ~(uint64_t)15;
                const uint4 v0 = *reinterpret_cast<const uint4 *>(W.wa);
                uint4 v1 = make_uint4(0, 0, 0, 0);
                if (W.wa + 16 < req_end) v1 = *reinterpret_cast<const uint4 *>(W.wa + 16);
                W.q0 = (uint64_t)v0.x | (uint64_t)v0.y << 32;
                W.q1 = (uint64_t)v0.z | (uint64_t)v0.w << 32;
                W.q2 = (uint64_t)v1.x | (uint64_t)v1.y << 32;
                W.q3 = (uint64_t)v1.z | (uint64_t)v1.w << 32;
                S.need = false;
            }
            // run until a window is needed, a second item is pending, or the end
            if (!S.done && !S.need)
                while (walk_step(S, W, b, q.version, s_prog)) {}
            // the client id: once every lane has read it (its first field)
            if (!client_done && !__any(!S.done && S.pc == prog_start(q.kind) && S.ms == M_NONE)) {
                client_done = true;
                int32_t cid = -2;
                if (walk && q.typed && S.client_len > 0) {
                    Cur cur;
                    cur.line = ~(uintptr_t)0;
                    cid = str_lookup(T.client_hash, T.client_mask, T.strings, cur, b + S.client_off, S.client_len);
                    if (cid < 0) cid = -2;
                }
                q.client = cid;
                Q.client[lane] = cid;
            }
            // queue this round's CRC items and topics (prefix by ballot; no atomics).
            // A lane whose item does not fit stops and is decoded again exactly.
            const uint64_t mc = __ballot(S.has_crc), mt = __ballot(S.has_topic);
            const uint32_t rc = __builtin_amdgcn_mbcnt_hi((uint32_t)(mc >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mc, 0));
            const uint32_t rt = __builtin_amdgcn_mbcnt_hi((uint32_t)(mt >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)mt, 0));
            if (S.has_crc) {
                if (nc + rc < kCrcQ && S.crc_len < (1u << 26)) {
                    Q.c_off[nc + rc] = S.crc_off;
                    Q.c_len[nc + rc] = S.crc_len | lane << 26;
                    Q.c_want[nc + rc] = S.crc_want;
                } else {
                    ovf = true;
                    S.done = true;
                }
                S.has_crc = false;
            }
            if (S.has_topic) {
                if (nt + rt < kTopQ) {
                    Q.t_off[nt + rt] = S.top_off;
                    Q.t_len[nt + rt] = S.top_len | lane << 26;
                } else {
                    ovf = true;
                    S.done = true;
                }
                S.has_topic = false;
            }
            nc = min(nc + (uint32_t)__builtin_popcountll(mc), kCrcQ);
            nt = min(nt + (uint32_t)__builtin_popcountll(mt), kTopQ);
        }
        // ---- the queued work: message CRCs, topic lookups
        __builtin_amdgcn_wave_barrier();
        KX_MARK(1);
        uint64_t bad = 0;  // request lanes with a mismatching CRC
        if (nc) bad = crc_pass(Q, nc, crctab, lane);
        KX_MARK(2);
        if (nt) flush_topics(T, Q, nt, lane);
        __builtin_amdgcn_wave_barrier();
        KX_MARK(3);
        if (walk) {
            if (ovf || ((bad >> lane) & 1)) {
                classify_exact(T, conn, b, len, crctab, r);
            } else if (S.rc == RS_ERROR || (S.rc == RS_OK && S.err)) {
                r.verdict = V_PARSE_ERROR;
                r.rule = -1;
                r.consumed = 0;
            } else if (S.rc == RS_COMPRESSED) {
                r.verdict = V_UNSUPPORTED;
                r.rule = -1;
                r.consumed = 0;
            } else {
                const DevKafkaRuleset rs = T.rulesets[conn.ruleset];
                match_rules(T, rs, q, q.typed == 1 ? S.ntopics : 0, Q.cmax[lane], rawlen, r);
            }
        }
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
        KX_MARK(4);
    }
    KX_FLUSH(lane);
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

#ifdef L7G_KX_TIMING
hipError_t KafkaPhaseTimes(uint64_t *out, bool reset) {
    hipError_t rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kx_phase), sizeof(unsigned long long) * 8);
    if (rc == hipSuccess && reset) {
        static const unsigned long long z[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        rc = hipMemcpyToSymbol(HIP_SYMBOL(g_kx_phase), z, sizeof z);
    }
    return rc;
}
#else
hipError_t KafkaPhaseTimes(uint64_t *, bool) { return hipErrorNotSupported; }
#endif

}  // namespace l7
