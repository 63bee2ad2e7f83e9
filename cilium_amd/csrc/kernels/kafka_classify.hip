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
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "kafka_dec.h"

namespace l7 {

namespace {

#ifndef L7G_KAFKA_BLOCK  // threads per workgroup: the CRC tables are shared by its waves
#define L7G_KAFKA_BLOCK 256
#endif
constexpr int kBlock = L7G_KAFKA_BLOCK;

// readMessageSet on the shared position; 0 ok, -1 error; zflag is set when a
// compressed message was passed
__device__ __forceinline__ int read_message_set(Cur &cur, const uint8_t *b, uint32_t &pos, uint32_t end, int32_t size,
                                int16_t version, const uint32_t *crctab, bool &zflag, uint8_t *stage) {
    if (size < 0) return 0;
    if ((uint32_t)size > kMaxParseBuf) return -1;
    KDec dec{b, pos, end, size, 0, &cur};
    int rc = 0;
    for (;;) {
        dec_skip(dec, 8);
        if (dec.err) break;
        int32_t msize = (int32_t)dec_int(dec, 4);
        if (dec.err || msize <= 0) break;
        if ((uint32_t)msize > kMaxParseBuf) { rc = -1; break; }
        uint32_t at = kread(dec, (uint32_t)msize);
        if (dec.err) break;
        KDec md{b, at, at + (uint32_t)msize, -1, 0, &cur};
        uint32_t crc = (uint32_t)dec_int(md, 4);
        if (msize <= 4) break;
        if (crc != crc32_ieee_staged(crctab, cur, b + at + 4, (uint32_t)msize - 4, stage)) break;  // stop, no drain
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


// 4 bytes at p as a little-endian word (bytes past a string's end are masked
// off by the caller)
__device__ __forceinline__ uint32_t le_load4(Cur &c, const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t k = (uint32_t)(a & 15);
    if (k <= 12) {
        cur_fill(c, a);
        const uint32_t w0 = c.w0, w1 = c.w1, w2 = c.w2, w3 = c.w3;
        const uint32_t i = k >> 2;
        const uint32_t lo = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
        const uint32_t hi = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
        return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
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
__device__ __forceinline__ int32_t str_lookup(const DevStrSlot *tab, uint32_t mask, const uint8_t *strings, Cur &cur,
                                              const uint8_t *s, uint32_t n) {
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

}  // namespace

// sel: this protocol's request indices from partition_kernel (mixed batches),
// else requests 0..n-1.  answer_other: answer entries on connections that are
// not Kafka (single-protocol engines, where partition_kernel does not run).
#ifndef L7G_KAFKA_WAVES
#define L7G_KAFKA_WAVES 6
#endif
#ifndef L7G_KAFKA_MAX_BLOCKS
#define L7G_KAFKA_MAX_BLOCKS 8192  // grid-stride beyond this (fixed-stride launches)
#endif
#ifndef L7G_KAFKA_DYN  // persistent grid, waves take 64 entries at a time from a per-launch counter
#define L7G_KAFKA_DYN 1
#endif
#ifndef L7G_KAFKA_GRIDMUL  // fixed-stride launches: grid = this many rounds of resident workgroups (0: L7G_KAFKA_MAX_BLOCKS cap)
#define L7G_KAFKA_GRIDMUL 0
#endif
#ifndef L7G_KAFKA_ORDER  // 1: the length classes longest first (the long requests start first, the short ones fill the tail)
#define L7G_KAFKA_ORDER 1
#endif
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(L7G_KAFKA_WAVES, 8))) void kafka_classify_kernel(
    Batch B, KafkaTables T, const uint32_t *__restrict__ sel, const uint32_t *__restrict__ sel_count,
    uint32_t answer_other, uint32_t *__restrict__ zlist, uint32_t *__restrict__ zcount, uint32_t *__restrict__ work) {
    const uint32_t n = B.n, nconns = B.nconns;
    const uint8_t *__restrict__ arena = B.arena;
    const uint32_t *__restrict__ conn_ids = B.conn_ids;
    const DevConn *__restrict__ conns = B.conns;
    static_assert(kBlock >= 256, "one CRC table entry per thread");
    __shared__ uint32_t crctab[kCrcTables * 256];
    // per wave: the CRC's 64-byte-per-lane staging area (crc32_ieee_staged)
    __shared__ __attribute__((aligned(16))) uint8_t crcstage[kBlock / 64][4096];
    uint8_t *stage = crcstage[threadIdx.x >> 6];
    crc_tables_init(crctab, threadIdx.x);
    // sel: this protocol's request indices from partition_kernel (mixed batches), else all n
    // (L7_KAFKA_CLASSES length classes, class c at sel + c * n, sel_count[c] entries each)
    constexpr int kCls = L7_KAFKA_CLASSES;
    uint32_t kc[kCls] = {n};
    uint32_t m = n;
    if (sel) {
        m = 0;
        for (int c = 0; c < kCls; c++) { kc[c] = sel_count[c]; m += kc[c]; }
    }
#if L7G_KAFKA_DYN
    // Entries after the grid's first sweep are taken 64 at a time (one per
    // lane) by whichever wave is free, from a per-launch counter the launcher
    // zeroes, so the persistent grid's waves finish together; else (no
    // counter) a fixed stride.  A lane whose entry is past the list end has no
    // later one either, so the loop may run divergent.
    const uint32_t stride = gridDim.x * kBlock;
    auto next_entry = [&](uint32_t i) -> uint32_t {
        if (!work) return i + stride;
        const uint32_t lane = threadIdx.x & 63;
        uint32_t t = 0;
        if (lane == (uint32_t)__builtin_amdgcn_readfirstlane(lane)) t = atomicAdd(work, 64u);
        return stride + __builtin_amdgcn_readfirstlane(t) + lane;
    };
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < m; i = next_entry(i)) {
#else
    for (uint32_t i = blockIdx.x * kBlock + threadIdx.x; i < m; i += gridDim.x * kBlock) {
#endif
        uint32_t idx = i;
        if (sel) {
#if L7G_KAFKA_ORDER == 1
            uint32_t c = kCls - 1, j = i;
            while (c > 0 && j >= kc[c]) { j -= kc[c]; c--; }
#else
            uint32_t c = 0, j = i;
            while (c < kCls - 1 && j >= kc[c]) { j -= kc[c]; c++; }
#endif
            idx = sel[(size_t)c * n + j];
        }
        const uint32_t ci = conn_ids[idx];
        const DevConn conn = ci < nconns ? conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
        const uint64_t off = B.offs[idx];
        const uint32_t len = B.lens[idx];
        const uint8_t *b = arena + off;
        Cur cur;
        cur.line = ~(uintptr_t)0;
        uint8_t verdict = V_PARSE_ERROR;
        int32_t rule = -1;
        uint32_t consumed = 0;
        bool zflag = false;  // compressed messages passed: kafka_inflate_kernel decides them
        if (conn.proto != PROTO_KAFKA || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
            if (!answer_other || (L7_PROTO_OWNED(conn.proto) && conn.proto != PROTO_KAFKA)) continue;
            verdict = V_UNSUPPORTED;  // unknown connection / no parser
        }
        // ---- proto.ReadReq
        do {
            if (verdict == V_UNSUPPORTED) break;
            if (!l7_in_arena(off, len, B.arena_len)) { verdict = V_UNSUPPORTED; break; }  // out of contract
            if (len < 4) { verdict = V_INCOMPLETE; break; }
            const int32_t size = (int32_t)be_load(cur, b, 4);
            if (size <= 0) { verdict = V_PARSE_ERROR; break; }
            if (len < 6) { verdict = V_INCOMPLETE; break; }
            if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) { verdict = V_PARSE_ERROR; break; }
            const uint32_t rawlen = (uint32_t)size + 4;
            if (rawlen > len) { verdict = V_INCOMPLETE; break; }
            if (rawlen < 12) { verdict = V_PARSE_ERROR; break; }
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
                KDec d{b, 0, rawlen, -1, 0, &cur};
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
                uint32_t o, l;
                switch (q.kind) {
                case 0:  // Produce
                    if (ver >= 3) dec_string(d, o, l);
                    dec_skip(d, 2); dec_skip(d, 4);
                    nt = dec_arraylen(d, false, bad);
                    if (bad) { rc = -1; break; }
                    for (int32_t t = 0; t < nt && rc == 0; t++) {
                        dec_string(d, o, l);
                        if (d.err) break;
                        on_topic(o, l);
                        np = dec_arraylen(d, false, bad);
                        if (bad) { rc = -1; break; }
                        for (int32_t p = 0; p < np; p++) {
                            dec_skip(d, 4);
                            if (d.err) { rc = -1; break; }
                            const int32_t ss = (int32_t)dec_int(d, 4);
                            if (d.err) { rc = -1; break; }
                            rc = read_message_set(cur, b, d.pos, d.end, ss, ver, crctab, zflag, stage);
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
                        dec_string(d, o, l);
                        on_topic(o, l);
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
                        dec_string(d, o, l);
                        on_topic(o, l);
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
                    for (int32_t t = 0; t < nt && !d.err; t++) { dec_string(d, o, l); if (!d.err) on_topic(o, l); }
                    if (ver >= 4) dec_skip(d, 1);
                    break;
                case 8:  // OffsetCommit
                    dec_string(d, o, l);
                    if (ver >= 1) { dec_skip(d, 4); dec_string(d, o, l); }
                    if (ver >= 2) dec_skip(d, 8);
                    nt = dec_arraylen(d, false, bad);
                    if (bad) { rc = -1; break; }
                    for (int32_t t = 0; t < nt && !d.err; t++) {
                        dec_string(d, o, l);
                        on_topic(o, l);
                        np = dec_arraylen(d, false, bad);
                        if (bad) { rc = -1; break; }
                        for (int32_t p = 0; p < np && !d.err; p++) {
                            dec_skip(d, 4); dec_skip(d, 8);
                            if (ver == 1) dec_skip(d, 8);
                            uint32_t o2, l2;
                            dec_string(d, o2, l2);
                        }
                    }
                    break;
                case 9:  // OffsetFetch
                    dec_string(d, o, l);
                    nt = dec_arraylen(d, true, bad);
                    if (bad) { rc = -1; break; }
                    for (int32_t t = 0; t < nt && !d.err; t++) {
                        dec_string(d, o, l);
                        on_topic(o, l);
                        np = dec_arraylen(d, false, bad);
                        if (bad) { rc = -1; break; }
                        for (int32_t p = 0; p < np && !d.err; p++) dec_skip(d, 4);
                    }
                    break;
                case 10:  // ConsumerMetadata
                    dec_string(d, o, l);
                    if (ver >= 1) dec_skip(d, 1);
                    break;
                }
                if (rc == 0 && d.err) rc = -1;
            }
            if (rc == -1) { verdict = V_PARSE_ERROR; break; }
            consumed = rawlen;
            verdict = V_DENY;
            if (!rs.any) break;
            // ---- MatchesRule
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
            if (best != kInf) { verdict = V_ALLOW; rule = T.rules[rs.rule_first + best].gid; }
        } while (false);
        B.verdict[idx] = verdict;
        B.rule[idx] = rule;
        B.consumed[idx] = consumed;
        if (zflag && zlist && (verdict == V_ALLOW || verdict == V_DENY)) zlist[atomicAdd(zcount, 1u)] = idx;
    }
}

hipError_t KafkaPhaseTimes(uint64_t *, bool) { return hipErrorNotSupported; }

hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, uint32_t *zlist, uint32_t *zcount, uint32_t *work,
                               hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
#if L7G_KAFKA_DYN
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
            resident = L7G_KAFKA_MAX_BLOCKS;
    }
    if (!work) blocks = blocks > L7G_KAFKA_MAX_BLOCKS ? L7G_KAFKA_MAX_BLOCKS : blocks;
    else if (blocks > (uint32_t)resident) blocks = (uint32_t)resident;
#else
    work = nullptr;
#if L7G_KAFKA_GRIDMUL
    static int resident = 0;
    if (resident == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess &&
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kafka_classify_kernel, kBlock, 0) == hipSuccess &&
            cus > 0 && per_cu > 0)
            resident = cus * per_cu * L7G_KAFKA_GRIDMUL;
        else
            resident = L7G_KAFKA_MAX_BLOCKS;
    }
    if (blocks > (uint32_t)resident) blocks = (uint32_t)resident;
#else
    if (blocks > L7G_KAFKA_MAX_BLOCKS) blocks = L7G_KAFKA_MAX_BLOCKS;
#endif
#endif
    hipLaunchKernelGGL(kafka_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                       answer_other ? 1u : 0u, zlist, zcount, work);
    return hipGetLastError();
}

}  // namespace l7
