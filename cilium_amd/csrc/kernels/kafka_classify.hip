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
// Round 4: the walk and the CRC no longer interleave.  kafka_classify_kernel
// walks each wave's 64 requests speculatively -- every message's CRC assumed
// to hold -- with a 64-byte register cursor (a message header, a topic entry,
// a request header: one memory latency each instead of two or three), and
// appends each message's CRC'd range to a per-wave list in LDS.  Then the
// wave's lanes take the listed messages one per lane and check their CRCs
// (kafka_dec.h slicing-by-8, all 64 lanes on the same code path).  A request
// whose messages all hold has exactly the reference's verdict (the walk the
// reference takes is the one taken); one with a mismatch -- where
// readMessageSet would have stopped the set without draining it and the walk
// gone on from there -- or with more messages than the wave's list holds is
// handed to kafka_exact_kernel, the lane-serial walk with the CRC in line
// (round 3's kernel), which decides it exactly.  Why: with the CRC inside the
// message loop a wave's lanes drifted apart (each lane's messages have other
// lengths), so the wave ran its lanes' header decodes and CRC batches one
// after the other, each behind its own memory latency (round 3: 74 % of wave
// cycles waiting, 2.9x refetch).
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "kafka_dec.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;
#ifndef L7G_KAFKA_CURW  // words the walk's register cursor holds (4, 8, 16: 16, 32, 64 bytes)
#define L7G_KAFKA_CURW 16
#endif
// message list of one wave: CRC'd range (request-relative start | lane), length, stored CRC
constexpr uint32_t kDescPerWave = 600;  // (4 waves' lists + the CRC tables: 40 KB, 4 workgroups per CU)
constexpr uint32_t kDescPosBits = 24;  // a request is at most kMaxParseBuf (< 2^23) bytes
static_assert(kMaxParseBuf < (1u << kDescPosBits), "message position field");

struct WaveDesc {
    uint32_t n;                    // appended (may exceed kDescPerWave: the overflowing lanes fall back)
    uint32_t bad;                  // bit l: lane l's request failed a CRC (lanes 0-31)
    uint32_t bad_hi;               // (lanes 32-63)
    uint32_t pad;
    uint64_t base[64];             // lane's request address
    uint32_t pos[kDescPerWave];    // CRC'd range start (request-relative) | lane << kDescPosBits
    uint32_t len[kDescPerWave];
    uint32_t crc[kDescPerWave];
};

// 4 bytes at p as a little-endian word (bytes past a string's end are masked
// off by the caller)
template <int NW>
__device__ __forceinline__ uint32_t le_load4(CurT<NW> &c, const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t k = (uint32_t)(a & (NW * 4 - 1));
    if (k <= NW * 4 - 4) {
        cur_fill(c, a);
        const uint32_t i = k >> 2;
        return __builtin_amdgcn_alignbyte(cur_wordi(c, i + 1), cur_wordi(c, i), k & 3);
    }
    uint32_t v = 0;
    for (int i = 0; i < 4; i++) v |= cur_byte(c, p + i) << (8 * i);
    return v;
}

// Interned id of the request string s[0, n) (topic or client id), -1 if the
// rule tables do not know it: word hash (l7_whash_*), linear probing, then a
// word-wise compare: the first 16 bytes against the slot's copy (the words
// were read for the hash), the rest against the 4-byte aligned, zero-padded
// table string.
template <int NW>
__device__ __forceinline__ int32_t str_lookup(const DevStrSlot *tab, uint32_t mask, const uint8_t *strings,
                                              CurT<NW> &cur, const uint8_t *s, uint32_t n) {
    uint32_t h = kWHashSeed;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;  // the first 16 bytes, zero-padded
    for (uint32_t i = 0; i < n; i += 4) {
        const uint32_t r = n - i;
        const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u;
        const uint32_t w = le_load4(cur, s + i) & keep;
        h = l7_whash_step(h, w);
        p0 = i == 0 ? w : p0;
        p1 = i == 4 ? w : p1;
        p2 = i == 8 ? w : p2;
        p3 = i == 12 ? w : p3;
    }
    h = l7_whash_final(h, n);
    for (uint32_t slot = h & mask;; slot = (slot + 1) & mask) {
        const DevStrSlot e = tab[slot];
        if (!e.used) return -1;
        if (e.hash == h && e.len == n) {
            bool eq = e.pre[0] == p0 && e.pre[1] == p1 && e.pre[2] == p2 && e.pre[3] == p3;
            const uint32_t *t = reinterpret_cast<const uint32_t *>(strings + e.str_off);
            for (uint32_t i = 16; i < n && eq; i += 4) {
                const uint32_t r = n - i;
                const uint32_t keep = r >= 4 ? 0xFFFFFFFFu : (1u << (8 * r)) - 1u;
                eq = t[i >> 2] == (le_load4(cur, s + i) & keep);
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
        const uint32_t w[6] = {e1.x, e1.y, e1.z, e1.w, e2.x, e2.y};
        __builtin_memcpy(&r0, w, sizeof r0);
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

// The per-message CRC check of readMessageSet, two ways.  Exact: computed in
// line, a mismatch stops the set.  Speculative: the message's CRC'd range is
// appended to the wave's list (checked after the walk) and the walk goes on
// as if it held; *spill is set when the list is full.
struct CrcExact {
    const uint32_t *crctab;
    uint8_t *stage;
    __device__ __forceinline__ bool holds(Cur &cur, const uint8_t *b, uint32_t at, uint32_t n, uint32_t crc) {
        return crc == crc32_ieee_staged(crctab, cur, b + at, n, stage);
    }
};
struct CrcDefer {
    WaveDesc *D;
    uint32_t lane;
    bool *spill;
    template <class C>
    __device__ __forceinline__ bool holds(C &, const uint8_t *, uint32_t at, uint32_t n, uint32_t crc) {
        const uint32_t k = atomicAdd(&D->n, 1u);
        if (k < kDescPerWave) {
            D->pos[k] = at | lane << kDescPosBits;
            D->len[k] = n;
            D->crc[k] = crc;
        } else {
            *spill = true;
        }
        return true;
    }
};

// readMessageSet on the shared position; 0 ok, -1 error; zflag is set when a
// compressed message was passed
template <class C, class CRC>
__device__ __forceinline__ int read_message_set(C &cur, const uint8_t *b, uint32_t &pos, uint32_t end, int32_t size,
                                                int16_t version, CRC &crcchk, bool &zflag) {
    if (size < 0) return 0;
    if ((uint32_t)size > kMaxParseBuf) return -1;
    KDecT<C> dec{b, pos, end, size, 0, &cur};
    int rc = 0;
    for (;;) {
        dec_skip(dec, 8);
        if (dec.err) break;
        int32_t msize = (int32_t)dec_int(dec, 4);
        if (dec.err || msize <= 0) break;
        if ((uint32_t)msize > kMaxParseBuf) { rc = -1; break; }
        uint32_t at = kread(dec, (uint32_t)msize);
        if (dec.err) break;
        KDecT<C> md{b, at, at + (uint32_t)msize, -1, 0, &cur};
        uint32_t crc = (uint32_t)dec_int(md, 4);
        if (msize <= 4) break;
        if (!crcchk.holds(cur, b, at + 4, (uint32_t)msize - 4, crc)) break;  // stop, no drain
        dec_skip(md, 1);
        int8_t attr = (int8_t)dec_int(md, 1);
        if (version >= 1) dec_skip(md, 8);
        int codec = attr & 3;
        if (codec == 3) break;  // `return nil, err` with err == nil
        dec_bytes(md);
        dec_bytes(md);
        if (md.err) { rc = -1; break; }
        // gzip / snappy: decoded (and its set read) by kafka_inflate_kernel;
        // the walk goes on, since a successful decode changes nothing here
        if (codec != 0) zflag = true;
    }
    pos = dec.pos;
    return rc;
}

// One request: proto.ReadReq, the typed decode, MatchesRule.
struct ReqOut {
    uint8_t verdict;
    int32_t rule;
    uint32_t consumed;
    bool zflag;
};
template <class C, class CRC>
__device__ __forceinline__ ReqOut classify_one(const Batch &B, const KafkaTables &T, uint32_t idx, uint32_t answer_other,
                                               bool &skip, C &cur, CRC &crcchk) {
    ReqOut o{V_PARSE_ERROR, -1, 0, false};
    skip = false;
    const uint32_t ci = B.conn_ids[idx];
    const DevConn conn = ci < B.nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    const uint64_t off = B.offs[idx];
    const uint32_t len = B.lens[idx];
    const uint8_t *b = B.arena + off;
    cur.line = ~(uintptr_t)0;
    if (conn.proto != PROTO_KAFKA || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
        if (!answer_other || (L7_PROTO_OWNED(conn.proto) && conn.proto != PROTO_KAFKA)) { skip = true; return o; }
        o.verdict = V_UNSUPPORTED;  // unknown connection / no parser
        return o;
    }
    // ---- proto.ReadReq
    if (!l7_in_arena(off, len, B.arena_len)) { o.verdict = V_UNSUPPORTED; return o; }  // out of contract
    if (len < 4) { o.verdict = V_INCOMPLETE; return o; }
    const int32_t size = (int32_t)be_load(cur, b, 4);
    if (size <= 0) { o.verdict = V_PARSE_ERROR; return o; }
    if (len < 6) { o.verdict = V_INCOMPLETE; return o; }
    if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) { o.verdict = V_PARSE_ERROR; return o; }
    const uint32_t rawlen = (uint32_t)size + 4;
    if (rawlen > len) { o.verdict = V_INCOMPLETE; return o; }
    if (rawlen < 12) { o.verdict = V_PARSE_ERROR; return o; }
    ReqInfo q;
    q.kind = (int16_t)be_load(cur, b + 4, 2);
    q.version = (int16_t)be_load(cur, b + 6, 2);
    q.typed = (q.kind == 0 || q.kind == 1 || q.kind == 2 || q.kind == 3 || q.kind == 8 || q.kind == 9) ? 1
            : (q.kind == 10 ? 2 : 0);
    q.client = -2;
    // fields are read where they are used: a copy would hold 9 VGPRs across the decode
    const DevKafkaRuleset &rs = T.rulesets[conn.ruleset];
    uint32_t ntopics = 0, cmax = 0;  // raw topic count; max over topics of first matching rule
    int rc = 0;
    if (q.typed) {
        KDecT<C> d{b, 0, rawlen, -1, 0, &cur};
        bool bad = false;
        dec_skip(d, 4); dec_skip(d, 2);
        const int16_t ver = (int16_t)dec_int(d, 2);
        dec_skip(d, 4);
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
        int32_t nt, np;
        uint32_t o2, l;
        switch (q.kind) {
        case 0:  // Produce
            if (ver >= 3) dec_string(d, o2, l);
            dec_skip(d, 2); dec_skip(d, 4);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && rc == 0; t++) {
                dec_string(d, o2, l);
                if (d.err) break;
                on_topic(o2, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = -1; break; }
                for (int32_t p = 0; p < np; p++) {
                    dec_skip(d, 4);
                    if (d.err) { rc = -1; break; }
                    const int32_t ss = (int32_t)dec_int(d, 4);
                    if (d.err) { rc = -1; break; }
                    rc = read_message_set(cur, b, d.pos, d.end, ss, ver, crcchk, o.zflag);
                    if (rc) break;
                }
            }
            break;
        case 1:  // Fetch
            dec_skip(d, 4); dec_skip(d, 4); dec_skip(d, 4);
            if (ver >= 3) dec_skip(d, 4);
            if (ver >= 4) dec_skip(d, 1);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o2, l);
                on_topic(o2, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = -1; break; }
                for (int32_t p = 0; p < np && !d.err; p++) {
                    dec_skip(d, 4); dec_skip(d, 8);
                    if (ver >= 5) dec_skip(d, 8);
                    dec_skip(d, 4);
                }
            }
            break;
        case 2:  // Offset
            dec_skip(d, 4);
            if (ver >= 2) dec_skip(d, 1);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o2, l);
                on_topic(o2, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = -1; break; }
                for (int32_t p = 0; p < np && !d.err; p++) {
                    dec_skip(d, 4); dec_skip(d, 8);
                    if (ver == 0) dec_skip(d, 4);
                }
            }
            break;
        case 3:  // Metadata
            nt = dec_arraylen(d, true, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && !d.err; t++) { dec_string(d, o2, l); if (!d.err) on_topic(o2, l); }
            if (ver >= 4) dec_skip(d, 1);
            break;
        case 8:  // OffsetCommit
            dec_string(d, o2, l);
            if (ver >= 1) { dec_skip(d, 4); dec_string(d, o2, l); }
            if (ver >= 2) dec_skip(d, 8);
            nt = dec_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o2, l);
                on_topic(o2, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = -1; break; }
                for (int32_t p = 0; p < np && !d.err; p++) {
                    dec_skip(d, 4); dec_skip(d, 8);
                    if (ver == 1) dec_skip(d, 8);
                    uint32_t o3, l3;
                    dec_string(d, o3, l3);
                }
            }
            break;
        case 9:  // OffsetFetch
            dec_string(d, o2, l);
            nt = dec_arraylen(d, true, bad);
            if (bad) { rc = -1; break; }
            for (int32_t t = 0; t < nt && !d.err; t++) {
                dec_string(d, o2, l);
                on_topic(o2, l);
                np = dec_arraylen(d, false, bad);
                if (bad) { rc = -1; break; }
                for (int32_t p = 0; p < np && !d.err; p++) dec_skip(d, 4);
            }
            break;
        case 10:  // ConsumerMetadata
            dec_string(d, o2, l);
            if (ver >= 1) dec_skip(d, 1);
            break;
        }
        if (rc == 0 && d.err) rc = -1;
    }
    if (rc == -1) { o.verdict = V_PARSE_ERROR; return o; }
    o.consumed = rawlen;
    o.verdict = V_DENY;
    if (!rs.any) return o;
    // ---- MatchesRule
    uint32_t best = kInf;
    if (ntopics == 0) {
        const int key = (q.kind >= 0 && q.kind < 64) ? q.kind : 64;
        const uint32_t koff = T.index[rs.bykey_off + 2 * key], cnt = T.index[rs.bykey_off + 2 * key + 1];
        for (uint32_t i = 0; i < cnt; i++) {
            uint32_t p = T.index[koff + i];
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
    if (best != kInf) { o.verdict = V_ALLOW; o.rule = T.rules[rs.rule_first + best].gid; }
    return o;
}

__device__ __forceinline__ void write_out(const Batch &B, uint32_t idx, const ReqOut &o, uint32_t *zlist,
                                          uint32_t *zcount) {
    B.verdict[idx] = o.verdict;
    B.rule[idx] = o.rule;
    B.consumed[idx] = o.consumed;
    if (o.zflag && zlist && (o.verdict == V_ALLOW || o.verdict == V_DENY)) zlist[atomicAdd(zcount, 1u)] = idx;
}

}  // namespace

// The speculative walk + CRC check over partition_kernel's Kafka lists
// (L7_KAFKA_CLASSES kind / length classes, class c at sel + c * n,
// sel_count[c] entries each; the longest class first), or requests 0..n-1
// when sel is null.  Waves take 64 entries at a time from work[0] (zeroed by
// the launcher).  Requests the walk cannot decide exactly are appended to
// fbl[k] (*fbn of them) for kafka_exact_kernel.  answer_other: answer
// entries on connections that are not Kafka (single-protocol engines).
__global__ __launch_bounds__(kBlock) void kafka_classify_kernel(Batch B, KafkaTables T, const uint32_t *__restrict__ sel,
                                                                const uint32_t *__restrict__ sel_count,
                                                                uint32_t answer_other, uint32_t *__restrict__ zlist,
                                                                uint32_t *__restrict__ zcount, uint32_t *__restrict__ work,
                                                                uint32_t *__restrict__ fbn, uint32_t *__restrict__ fbl) {
    const uint32_t n = B.n;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    static_assert(kBlock >= 256, "one CRC table entry per thread");
    __shared__ uint32_t crctab[kCrcTables * 256];
    __shared__ WaveDesc wdesc[kWaves];
    WaveDesc *D = &wdesc[wave];
    crc_tables_init(crctab, threadIdx.x);
    const uint32_t tabaddr = (uint32_t)(uintptr_t)crctab;
    constexpr int kCls = L7_KAFKA_CLASSES;
    uint32_t kc[kCls];
    uint32_t m = n;
    if (sel) {
        m = 0;
#pragma unroll
        for (int c = 0; c < kCls; c++) { kc[c] = sel_count[c]; m += kc[c]; }
    }
    for (;;) {
        uint32_t t0 = 0;
        if (lane == 0) t0 = atomicAdd(work, 64u);
        const uint32_t base = __builtin_amdgcn_readfirstlane(__shfl(t0, 0));
        if (base >= m) break;
        if (lane == 0) { D->n = 0; D->bad = 0; D->bad_hi = 0; }
        // (one wave's LDS operations complete in order: the other lanes see these)
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // ---- the walk (speculative: every CRC assumed to hold)
        const uint32_t i = base + lane;
        uint32_t idx = 0;
        ReqOut o{V_PARSE_ERROR, -1, 0, false};
        bool skip = true, spill = false;
        if (i < m) {
            idx = i;
            if (sel) {  // the length classes longest first (the long requests start first)
                uint32_t c = kCls - 1, j = i;
#pragma unroll
                for (int cc = kCls - 1; cc > 0; cc--)
                    if (c == (uint32_t)cc && j >= kc[cc]) { j -= kc[cc]; c = cc - 1; }
                idx = sel[(size_t)c * n + j];
            }
            D->base[lane] = (uint64_t)(uintptr_t)(B.arena + B.offs[idx]);
            CurT<L7G_KAFKA_CURW> cur;
            CrcDefer dc{D, lane, &spill};
            o = classify_one(B, T, idx, answer_other, skip, cur, dc);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // ---- the listed messages' CRCs, one message per lane
        const uint32_t nd = min(__builtin_amdgcn_readfirstlane(D->n), kDescPerWave);
        for (uint32_t k = lane; k < nd; k += 64) {
            const uint32_t pw = D->pos[k];
            const uint32_t owner = pw >> kDescPosBits;
            const uint8_t *p = (const uint8_t *)(uintptr_t)D->base[owner] + (pw & ((1u << kDescPosBits) - 1));
#ifdef KEXP_NOCRCPH
            if (D->len[k] == 0xFFFFFFFFu)
#else
            if (crc32_ieee_global(tabaddr, p, D->len[k]) != D->crc[k])
#endif
                atomicOr(owner < 32 ? &D->bad : &D->bad_hi, 1u << (owner & 31));
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        // ---- answer, or hand over to the exact walk
        if (i < m && !skip) {
            const uint32_t badw = lane < 32 ? D->bad : D->bad_hi;
            if (spill || ((badw >> (lane & 31)) & 1)) fbl[atomicAdd(fbn, 1u)] = idx;
            else write_out(B, idx, o, zlist, zcount);
        }
    }
}

// The exact lane-serial walk (CRC in line) over the handed-over list.
__global__ __launch_bounds__(kBlock) void kafka_exact_kernel(Batch B, KafkaTables T, const uint32_t *__restrict__ fbn,
                                                             const uint32_t *__restrict__ fbl, uint32_t answer_other,
                                                             uint32_t *__restrict__ zlist, uint32_t *__restrict__ zcount) {
    __shared__ uint32_t crctab[kCrcTables * 256];
    // per wave: the CRC's 64-byte-per-lane staging area (crc32_ieee_staged)
    __shared__ __attribute__((aligned(16))) uint8_t crcstage[kBlock / 64][4096];
    crc_tables_init(crctab, threadIdx.x);
    const uint32_t m = *fbn;
    CrcExact ce{crctab, crcstage[threadIdx.x >> 6]};
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
        const uint32_t idx = fbl[i];
        Cur cur;
        bool skip;
        const ReqOut o = classify_one(B, T, idx, answer_other, skip, cur, ce);
        if (!skip) write_out(B, idx, o, zlist, zcount);
    }
}

hipError_t KafkaPhaseTimes(uint64_t *, bool) { return hipErrorNotSupported; }

// work: the entry counter and fbn the hand-over count (both zeroed by the
// caller on `stream`); fbl: n words.
hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, uint32_t *zlist, uint32_t *zcount, uint32_t *work, uint32_t *fbn,
                               uint32_t *fbl, hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    if (!work || !fbn || !fbl) return hipErrorInvalidValue;
    // persistent grid: as many workgroups as the CUs hold at once
    static int resident = 0;
    if (resident == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kafka_classify_kernel, kBlock, 0) == hipSuccess &&
            cus > 0 && per_cu > 0)
            resident = cus * per_cu;
        else
            resident = 1024;
    }
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
    if (blocks > (uint32_t)resident) blocks = (uint32_t)resident;
    hipLaunchKernelGGL(kafka_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                       answer_other ? 1u : 0u, zlist, zcount, work, fbn, fbl);
    hipError_t rc = hipGetLastError();
    if (rc != hipSuccess) return rc;
    // the requests handed over (a CRC mismatch, a message list overflow): usually none,
    // so a small grid that reads the count and exits
    hipLaunchKernelGGL(kafka_exact_kernel, dim3(64), dim3(kBlock), 0, stream, B, T, fbn, fbl, answer_other ? 1u : 0u,
                       zlist, zcount);
    return hipGetLastError();
}

}  // namespace l7
