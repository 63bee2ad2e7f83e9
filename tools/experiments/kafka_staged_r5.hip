// Kafka request classification on gfx950 (product code).
//
// The decode path restated is the reference's: proto.ReadReq framing
// (vendor/github.com/optiopay/kafka/proto/messages.go:124-165), the typed
// decoders (:504-537, :767-824, :1033-1054, :1173-1228, :1389-1430,
// :1591-1647, :1810-1858) with io.ReadFull / LimitReader semantics
// (serialization.go:19-203), readMessageSet with CRC32-IEEE per message and
// stop-without-drain (:363-494), then MatchesRule (pkg/kafka/policy.go:200-225)
// against the connection's rule set using the precomputed topic / key views
// (engine/kafka_compile.h).  Requests with compressed messages are listed for
// kafka_inflate_kernel (kafka_inflate.hip), which decodes them.
//
// How the work is laid out (round 5).  A wave takes 64 list entries at a time
// and cuts them into sub-batches whose bytes fit its LDS buffer (kCap).  Per
// sub-batch:
//   1. stage: the requests' 16-byte chunks are copied HBM -> LDS by LDS-DMA,
//      64 chunks per instruction, every lane busy whatever the request
//      lengths (chunk -> request by a ballot over the chunk-start flags);
//      every request byte is read from HBM once, in whole lines;
//   2. walk: one lane per request decodes its request from LDS with the
//      reference's decoders, assuming every message CRC holds; it records each
//      message (CRC input, stored CRC) and each topic string instead of
//      checking / looking them up on the spot;
//   3. lookups: the client ids (a lane per request) and then the recorded
//      topics (a lane per topic) go to the hash tables in HBM together, so a
//      sub-batch waits two or three table round trips, not that many per
//      topic of each request;
//   4. CRC: every recorded message is cut into 36-byte segments aligned on its
//      end; a lane per segment computes raw(0, segment) as the XOR of 72
//      nibble-table reads (16-entry tables sit in 16 distinct LDS banks, so no
//      read ever conflicts), shifts it to the message end with power-of-two
//      zero-byte tables and XORs it into the message's accumulator
//      (crc(M) = ~XOR_j shift(raw(0, S_j)), the initial register folded into
//      the first four bytes);
//   5. a request any of whose messages fails its CRC (or that overflowed a
//      list, or a message shorter than 4 bytes) is redone by the exact
//      lane-serial path below, which stops at the failing message as the
//      reference does; otherwise MatchesRule decides it.
// Requests too long for the buffer, and entries that are not Kafka, take the
// exact path directly.  Every verdict is bit-exact either way: the deferred
// walk equals the exact one whenever every message it reached has a good CRC,
// and it records every message it reaches.
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "kafka_dec.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;
constexpr int kWaves = kBlock / 64;

// ---------------- CRC32-IEEE nibble tables (built at compile time) ----------------
// T_p[b] = raw(0, b . 0^p): the CRC register after byte b followed by p zero
// bytes, from state 0.  raw is linear in the bytes, so T_p[b] = T_p[b & 15] ^
// T_p[b & 0xF0]: nib[p][h][v] = T_p[v << 4h].  z[s][k][v] = raw(v << 4k,
// 0^(36 * 2^s)): the register shifted past 36 * 2^s zero bytes, nibble k of
// the state at a time.
constexpr int kSeg = 36;        // bytes per CRC segment
constexpr int kShiftTabs = 8;   // shifts by 36 * 2^s, s < 8 (messages up to 9 KiB)
struct CrcNib {
    uint32_t nib[kSeg][2][16];
    uint32_t z[kShiftTabs][8][16];
};
constexpr CrcNib make_crc_nib() {
    CrcNib t{};
    uint32_t t0[256] = {};
    for (uint32_t b = 0; b < 256; b++) {
        uint32_t c = b;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        t0[b] = c;
    }
    for (int h = 0; h < 2; h++)
        for (uint32_t v = 0; v < 16; v++) {
            uint32_t c = t0[v << (4 * h)];
            for (int p = 0; p < kSeg; p++) {
                t.nib[p][h][v] = c;
                c = (c >> 8) ^ t0[c & 0xFF];
            }
        }
    for (int k = 0; k < 8; k++)
        for (uint32_t v = 0; v < 16; v++) {
            uint32_t c = v << (4 * k);
            for (int i = 0; i < kSeg; i++) c = (c >> 8) ^ t0[c & 0xFF];
            t.z[0][k][v] = c;
        }
    for (int s = 1; s < kShiftTabs; s++)
        for (int k = 0; k < 8; k++)
            for (uint32_t v = 0; v < 16; v++) {
                uint32_t c = v << (4 * k);
                for (int rep = 0; rep < 2; rep++) {
                    uint32_t r = 0;
                    for (int j = 0; j < 8; j++) r ^= t.z[s - 1][j][(c >> (4 * j)) & 15];
                    c = r;
                }
                t.z[s][k][v] = c;
            }
    return t;
}
__constant__ CrcNib kCrcNib = make_crc_nib();
constexpr uint32_t kTabBytes = sizeof(CrcNib);  // 8704
static_assert(kTabBytes % 16 == 0, "table block alignment");
constexpr uint32_t kNibOff = 0, kZOff = sizeof(uint32_t) * kSeg * 2 * 16;

// ---------------- per-wave LDS layout ----------------
#ifndef L7G_KAFKA_CAP
#define L7G_KAFKA_CAP 6144
#endif
constexpr uint32_t kCap = L7G_KAFKA_CAP;  // request bytes staged per sub-batch
static_assert(kCap % 1024 == 0 && kCap <= 9216, "one DMA instruction stages 1 KiB; shifts cover 9 KiB");
constexpr uint32_t kCapChunks = kCap / 16;
constexpr uint32_t kMaxMsgs = 128, kMaxSegs = 384, kMaxTopics = 256;
constexpr uint32_t al4(uint32_t x) { return (x + 3) & ~3u; }
constexpr uint32_t W_BUF = 64;                         // 64-byte guard before the requests
constexpr uint32_t W_MA = W_BUF + kCap + 64;           // u16 CRC input start (buffer offset)
constexpr uint32_t W_ML = W_MA + 2 * kMaxMsgs;         // u16 CRC input length
constexpr uint32_t W_MS = W_ML + 2 * kMaxMsgs;         // u16 first segment
constexpr uint32_t W_MO = W_MS + 2 * kMaxMsgs;         // u8 owner lane
constexpr uint32_t W_MC = al4(W_MO + kMaxMsgs);        // u32 stored CRC
constexpr uint32_t W_MX = W_MC + 4 * kMaxMsgs;         // u32 accumulator
constexpr uint32_t W_TR = W_MX + 4 * kMaxMsgs;         // u32 topic record: pos | len << 14 | lane << 22
constexpr uint32_t W_CF = W_TR + 4 * kMaxTopics;       // u8 chunk starts: owner lane + 1
constexpr uint32_t W_SF = W_CF + kCapChunks;           // u8 segment starts: message + 1
constexpr uint32_t W_LR = al4(W_SF + kMaxSegs);        // i32 rule set, per lane
constexpr uint32_t W_LQ = W_LR + 256;                  // u32 kind | version << 16, per lane
constexpr uint32_t W_LC = W_LQ + 256;                  // i32 interned client id, per lane
constexpr uint32_t W_LM = W_LC + 256;                  // u32 max over topics of the first matching rule
constexpr uint32_t W_CTR = W_LM + 256;                 // u32 messages << 16 | segments
constexpr uint32_t W_NT = W_CTR + 4;                   // u32 topics
constexpr uint32_t W_BAD = W_NT + 4;                   // u32[2] lanes whose CRC failed
constexpr uint32_t kWaveBytes = (W_BAD + 8 + 15) & ~15u;
constexpr uint32_t kLdsBytes = kTabBytes + kWaves * kWaveBytes;
static_assert((W_CF - W_TR) % 4 == 0 && (W_SF + kMaxSegs - W_CF) % 8 == 0, "flag clearing in words");
static_assert(kCap + 64 < (1u << 14), "topic record position field");

__device__ __forceinline__ uint32_t bswap(uint32_t x) { return __builtin_amdgcn_perm(0, x, 0x00010203u); }
__device__ __forceinline__ uint32_t lds32(const uint8_t *lds, uint32_t a) {
    return *reinterpret_cast<const uint32_t *>(lds + a);
}
// little-endian 4 bytes at LDS byte offset a (any alignment)
__device__ __forceinline__ uint32_t lds_le4(const uint8_t *lds, uint32_t a) {
    const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + (a & ~3u));
    return __builtin_amdgcn_alignbyte(w[1], w[0], a & 3);
}
__device__ __forceinline__ void wave_sync() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_wave_barrier();
}

// raw(0, x[0..35]) from the nibble tables: no serial chain
__device__ __forceinline__ uint32_t seg_raw(const uint8_t *lds, const uint32_t (&x)[9]) {
    uint32_t r0 = 0, r1 = 0;
#pragma unroll
    for (int i = 0; i < 9; i++) {
        const uint32_t lo = (x[i] & 0x0F0F0F0Fu) << 2, hi = (x[i] >> 2) & 0x3C3C3C3Cu;
#pragma unroll
        for (int b = 0; b < 4; b++) {
            const uint32_t p = kSeg - 1 - (4 * i + b);
            r0 ^= lds32(lds, kNibOff + (2 * p) * 64 + ((lo >> (8 * b)) & 0xFF));
            r1 ^= lds32(lds, kNibOff + (2 * p + 1) * 64 + ((hi >> (8 * b)) & 0xFF));
        }
    }
    return r0 ^ r1;
}
// the register shifted past 36 * 2^s zero bytes
__device__ __forceinline__ uint32_t crc_shift(const uint8_t *lds, uint32_t s, uint32_t c) {
    const uint32_t base = kZOff + s * 512;
    const uint32_t lo = (c & 0x0F0F0F0Fu) << 2, hi = (c >> 2) & 0x3C3C3C3Cu;
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 4; b++)
        r ^= lds32(lds, base + (2 * b) * 64 + ((lo >> (8 * b)) & 0xFF)) ^
             lds32(lds, base + (2 * b + 1) * 64 + ((hi >> (8 * b)) & 0xFF));
    return r;
}
// one byte through the register: T_0[(c ^ b) & 0xFF] ^ (c >> 8)
__device__ __forceinline__ uint32_t crc_byte(const uint8_t *lds, uint32_t c, uint32_t b) {
    const uint32_t x = (c ^ b) & 0xFF;
    return (c >> 8) ^ lds32(lds, kNibOff + ((x & 15) << 2)) ^ lds32(lds, kNibOff + 64 + ((x >> 4) << 2));
}
// eight bytes (lo ^ c, hi) through the register: XOR of T_{7-k}[byte k]
__device__ __forceinline__ uint32_t crc_step8n(const uint8_t *lds, uint32_t lo, uint32_t hi) {
    uint32_t r = 0;
#pragma unroll
    for (int b = 0; b < 4; b++) {
        const uint32_t xl = (lo >> (8 * b)) & 0xFF, xh = (hi >> (8 * b)) & 0xFF;
        const uint32_t pl = 7 - b, ph = 3 - b;
        r ^= lds32(lds, kNibOff + (2 * pl) * 64 + ((xl & 15) << 2)) ^
             lds32(lds, kNibOff + (2 * pl + 1) * 64 + ((xl >> 4) << 2)) ^
             lds32(lds, kNibOff + (2 * ph) * 64 + ((xh & 15) << 2)) ^
             lds32(lds, kNibOff + (2 * ph + 1) * 64 + ((xh >> 4) << 2));
    }
    return r;
}

// ---------------- byte sources ----------------
// 4 bytes at p as a little-endian word through the lane's global chunk cursor
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
// the request in HBM (exact path)
struct GRd {
    static constexpr bool kLds = false;
    const uint8_t *b;
    Cur cur;
    __device__ __forceinline__ uint32_t le4(uint32_t pos) { return le_load4(cur, b + pos); }
    __device__ __forceinline__ uint64_t be(uint32_t pos, int n) { return be_load(cur, b + pos, n); }
};
// the request staged in LDS (deferred path): byte 0 at LDS offset at
struct LRd {
    static constexpr bool kLds = true;
    const uint8_t *lds;
    uint32_t at;
    __device__ __forceinline__ uint32_t le4(uint32_t pos) { return lds_le4(lds, at + pos); }
    // bytes [pos, pos + 36) as little-endian words, in one round of LDS reads
    __device__ __forceinline__ void win9(uint32_t pos, uint32_t (&x)[9]) {
        const uint32_t a = at + pos;
        const uint32_t *w = reinterpret_cast<const uint32_t *>(lds + (a & ~3u));
        uint32_t v[10];
#pragma unroll
        for (int i = 0; i < 10; i++) v[i] = w[i];
#pragma unroll
        for (int i = 0; i < 9; i++) x[i] = __builtin_amdgcn_alignbyte(v[i + 1], v[i], a & 3);
    }
    __device__ __forceinline__ uint64_t be(uint32_t pos, int n) {
        if (n == 8) return (uint64_t)bswap(le4(pos)) << 32 | bswap(le4(pos + 4));
        const uint32_t v = bswap(le4(pos));
        return n == 4 ? v : v >> (32 - 8 * n);
    }
};

// ---------------- io.ReadFull / LimitReader decoding over a byte source ----------------
template <class R>
struct KD {
    R *r;
    uint32_t pos, end;
    int32_t limit;  // LimitReader remaining, -1 = none
    int err;        // 0 ok, 1 EOF, 2 ErrUnexpectedEOF, 3 other
};
template <class R>
__device__ __forceinline__ uint32_t kd_read(KD<R> &d, uint32_t n) {
    const uint32_t at = d.pos;
    if (n == 0) return at;
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint32_t)d.limit < a) a = (uint32_t)d.limit;
    if (a == 0) { d.err = 1; return at; }
    const uint32_t take = a < n ? a : n;
    d.pos += take;
    if (d.limit >= 0) d.limit -= (int32_t)take;
    if (take < n) d.err = 2;
    return at;
}
template <class R>
__device__ __forceinline__ int64_t kd_int(KD<R> &d, int n) {
    if (d.err) return 0;
    const uint32_t at = kd_read(d, (uint32_t)n);
    if (d.err) return 0;
    const uint64_t v = d.r->be(at, n);
    return n == 1 ? (int64_t)(int8_t)v : n == 2 ? (int64_t)(int16_t)v : n == 4 ? (int64_t)(int32_t)v : (int64_t)v;
}
template <class R>
__device__ __forceinline__ void kd_skip(KD<R> &d, int n) {
    if (d.err) return;
    kd_read(d, (uint32_t)n);
}
template <class R>
__device__ __forceinline__ void kd_string(KD<R> &d, uint32_t &off, uint32_t &len) {  // DecodeString; len < 1 => ""
    off = 0; len = 0;
    if (d.err) return;
    const int16_t sl = (int16_t)kd_int(d, 2);
    if (d.err || sl < 1) return;
    const uint32_t at = kd_read(d, (uint32_t)sl);
    if (d.err) return;
    off = at; len = (uint32_t)sl;
}
template <class R>
__device__ __forceinline__ int32_t kd_arraylen(KD<R> &d, bool nullable, bool &bad) {  // DecodeArrayLen
    const int32_t l = (int32_t)kd_int(d, 4);
    bad = false;
    if (l < 0) { if (nullable) return -1; bad = true; return 0; }
    if ((uint32_t)l > kMaxParseBuf) { bad = true; return 0; }
    return l;
}
// np fixed-size entries whose fields are all skipped: passed in one step when
// they all lie inside the input (the per-field loop then cannot fail)
template <class R>
__device__ __forceinline__ bool kd_bulk(KD<R> &d, int32_t np, uint32_t esize) {
    if (d.err || np < 0) return false;
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint32_t)d.limit < a) a = (uint32_t)d.limit;
    const uint64_t need = (uint64_t)(uint32_t)np * esize;
    if (need > a) return false;
    d.pos += (uint32_t)need;
    if (d.limit >= 0) d.limit -= (int32_t)need;
    return true;
}
template <class R>
__device__ __forceinline__ void kd_bytes(KD<R> &d) {
    if (d.err) return;
    const int32_t sl = (int32_t)kd_int(d, 4);
    if (d.err || sl < 1) return;
    if ((uint32_t)sl > kMaxParseBuf) { d.err = 3; return; }
    kd_read(d, (uint32_t)sl);
}

// readMessageSet (messages.go:363-494) on the shared position; 0 ok, -1 error.
// h.msg(pos, len, stored) answers whether the CRC of the message's bytes
// [pos, pos + len) equals stored; false stops the set without draining it.
template <class R, class H>
__device__ __forceinline__ int kd_message_set(R &r, uint32_t &pos, uint32_t end, int32_t size, int16_t version,
                                              bool &zflag, H &h) {
    if (size < 0) return 0;
    if ((uint32_t)size > kMaxParseBuf) return -1;
    KD<R> dec{&r, pos, end, size, 0};
    int rc = 0;
    if constexpr (R::kLds) {
        // Messages whose header, key and value all lie inside the message and
        // the set take this path: one 36-byte window read per message (offset,
        // size, CRC, magic, attributes, [timestamp,] key length and, with no
        // key, value length), the fields at fixed places.  It takes exactly the
        // steps of the loop below and commits a message only when every one of
        // them succeeds; anything else goes to that loop, from the same message.
        const uint32_t hmin = version >= 1 ? 22u : 14u;  // crc magic attr [ts] klen vlen
        for (;;) {
            uint32_t avail = dec.end - dec.pos;
            if ((uint32_t)dec.limit < avail) avail = (uint32_t)dec.limit;
            if (avail < 12 + hmin) break;
            uint32_t x[9];
            r.win9(dec.pos, x);
            const uint32_t msize = bswap(x[2]);
            if ((int32_t)msize < (int32_t)hmin || 12 + msize > avail) break;
            const uint32_t at = dec.pos + 12;
            const uint32_t crc = bswap(x[3]);
            const uint32_t attr = (x[4] >> 8) & 0xFF;
            const int32_t klen = (int32_t)bswap(version >= 1 ? __builtin_amdgcn_alignbyte(x[7], x[6], 2)
                                                             : __builtin_amdgcn_alignbyte(x[5], x[4], 2));
            const uint32_t ko = at + (version >= 1 ? 14u : 6u);  // key length field
            uint32_t vo = ko + 4;
            int32_t vlen;
            if (klen < 1) {
                vlen = (int32_t)bswap(version >= 1 ? __builtin_amdgcn_alignbyte(x[8], x[7], 2)
                                                   : __builtin_amdgcn_alignbyte(x[6], x[5], 2));
            } else {
                if ((uint32_t)klen > msize || vo + (uint32_t)klen + 4 > at + msize) break;
                vo += (uint32_t)klen;
                vlen = (int32_t)r.be(vo, 4);
            }
            if (vlen >= 1 && ((uint32_t)vlen > msize || vo + 4 + (uint32_t)vlen > at + msize)) break;
            // committed: the message is read whole
            dec.pos = at + msize;
            dec.limit -= (int32_t)(12 + msize);
            if (!h.msg(at + 4, msize - 4, crc)) { pos = dec.pos; return 0; }  // stop, no drain
            if ((attr & 3) == 3) { pos = dec.pos; return 0; }
            if (attr & 3) zflag = true;
        }
    }
    for (;;) {
        kd_skip(dec, 8);
        if (dec.err) break;
        const int32_t msize = (int32_t)kd_int(dec, 4);
        if (dec.err || msize <= 0) break;
        if ((uint32_t)msize > kMaxParseBuf) { rc = -1; break; }
        const uint32_t at = kd_read(dec, (uint32_t)msize);
        if (dec.err) break;
        KD<R> md{&r, at, at + (uint32_t)msize, -1, 0};
        const uint32_t crc = (uint32_t)kd_int(md, 4);
        if (msize <= 4) break;
        if (!h.msg(at + 4, (uint32_t)msize - 4, crc)) break;  // stop, no drain
        kd_skip(md, 1);
        const int8_t attr = (int8_t)kd_int(md, 1);
        if (version >= 1) kd_skip(md, 8);
        const int codec = attr & 3;
        if (codec == 3) break;  // `return nil, err` with err == nil
        kd_bytes(md);
        kd_bytes(md);
        if (md.err) { rc = -1; break; }
        // gzip / snappy: decoded (and its set read) by kafka_inflate_kernel;
        // the walk goes on, since a successful decode changes nothing here
        if (codec != 0) zflag = true;
    }
    pos = dec.pos;
    return rc;
}

__device__ __forceinline__ bool is_topic_api_key(int k) {
    // 0 1 2 3 4 5 6 8 9 19 20 21 23 24 27 28 34 35 37
    if (k < 0 || k > 37) return false;
    const uint64_t m = (1ull << 0) | (1ull << 1) | (1ull << 2) | (1ull << 3) | (1ull << 4) | (1ull << 5) | (1ull << 6) |
                       (1ull << 8) | (1ull << 9) | (1ull << 19) | (1ull << 20) | (1ull << 21) | (1ull << 23) |
                       (1ull << 24) | (1ull << 27) | (1ull << 28) | (1ull << 34) | (1ull << 35) | (1ull << 37);
    return (m >> k) & 1;
}
__device__ __forceinline__ int kind_typed(int kind) {  // 0 nil request, 1 typed with topics/ClientID, 2 ConsumerMetadata
    return (kind == 0 || kind == 1 || kind == 2 || kind == 3 || kind == 8 || kind == 9) ? 1 : (kind == 10 ? 2 : 0);
}

// The typed decoders of one request after its frame checks (kinds 0 1 2 3 8 9
// 10); h.client(off, len) gets the ClientID, h.topic(off, len) each topic
// string in wire order.  0 ok, -1 error.
template <class R, class H>
__device__ __forceinline__ int kafka_walk(R &r, uint32_t rawlen, int kind, bool &zflag, H &h) {
    KD<R> d{&r, 0, rawlen, -1, 0};
    bool bad = false;
    int rc = 0;
    kd_skip(d, 4); kd_skip(d, 2);
    const int16_t ver = (int16_t)kd_int(d, 2);
    kd_skip(d, 4);
    uint32_t co, cl;
    kd_string(d, co, cl);
    if (!d.err && cl > 0) h.client(co, cl);
    int32_t nt, np;
    uint32_t o, l;
    switch (kind) {
    case 0:  // Produce
        if (ver >= 3) kd_string(d, o, l);
        kd_skip(d, 2); kd_skip(d, 4);
        nt = kd_arraylen(d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && rc == 0; t++) {
            kd_string(d, o, l);
            if (d.err) break;
            h.topic(o, l);
            np = kd_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np; p++) {
                kd_skip(d, 4);
                if (d.err) { rc = -1; break; }
                const int32_t ss = (int32_t)kd_int(d, 4);
                if (d.err) { rc = -1; break; }
                rc = kd_message_set(r, d.pos, d.end, ss, ver, zflag, h);
                if (rc) break;
            }
        }
        break;
    case 1:  // Fetch
        kd_skip(d, 4); kd_skip(d, 4); kd_skip(d, 4);
        if (ver >= 3) kd_skip(d, 4);
        if (ver >= 4) kd_skip(d, 1);
        nt = kd_arraylen(d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(d, o, l);
            h.topic(o, l);
            np = kd_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            if (kd_bulk(d, np, ver >= 5 ? 24u : 16u)) continue;
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
        nt = kd_arraylen(d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(d, o, l);
            h.topic(o, l);
            np = kd_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            if (kd_bulk(d, np, ver == 0 ? 16u : 12u)) continue;
            for (int32_t p = 0; p < np && !d.err; p++) {
                kd_skip(d, 4); kd_skip(d, 8);
                if (ver == 0) kd_skip(d, 4);
            }
        }
        break;
    case 3:  // Metadata
        nt = kd_arraylen(d, true, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(d, o, l);
            if (!d.err) h.topic(o, l);
        }
        if (ver >= 4) kd_skip(d, 1);
        break;
    case 8:  // OffsetCommit
        kd_string(d, o, l);
        if (ver >= 1) { kd_skip(d, 4); kd_string(d, o, l); }
        if (ver >= 2) kd_skip(d, 8);
        nt = kd_arraylen(d, false, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(d, o, l);
            h.topic(o, l);
            np = kd_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            for (int32_t p = 0; p < np && !d.err; p++) {
                kd_skip(d, 4); kd_skip(d, 8);
                if (ver == 1) kd_skip(d, 8);
                uint32_t o2, l2;
                kd_string(d, o2, l2);
            }
        }
        break;
    case 9:  // OffsetFetch
        kd_string(d, o, l);
        nt = kd_arraylen(d, true, bad);
        if (bad) { rc = -1; break; }
        for (int32_t t = 0; t < nt && !d.err; t++) {
            kd_string(d, o, l);
            h.topic(o, l);
            np = kd_arraylen(d, false, bad);
            if (bad) { rc = -1; break; }
            if (kd_bulk(d, np, 4u)) continue;
            for (int32_t p = 0; p < np && !d.err; p++) kd_skip(d, 4);
        }
        break;
    case 10:  // ConsumerMetadata
        kd_string(d, o, l);
        if (ver >= 1) kd_skip(d, 1);
        break;
    }
    if (rc == 0 && d.err) rc = -1;
    return rc;
}

// Interned id of the request string at [pos, pos + n) (topic or client id),
// -1 if the rule tables do not know it: word hash (l7_whash_*), linear
// probing, then a word-wise compare: the first 16 bytes against the slot's
// copy (the words were read for the hash), the rest against the 4-byte
// aligned, zero-padded table string.
template <class R>
__device__ __forceinline__ int32_t str_lookup(const DevStrSlot *tab, uint32_t mask, const uint8_t *strings, R &r,
                                              uint32_t pos, uint32_t n) {
    uint32_t h = kWHashSeed;
    uint32_t p0 = 0, p1 = 0, p2 = 0, p3 = 0;  // the first 16 bytes, zero-padded
    for (uint32_t i = 0; i < n; i += 4) {
        const uint32_t rem = n - i;
        const uint32_t keep = rem >= 4 ? 0xFFFFFFFFu : (1u << (8 * rem)) - 1u;
        const uint32_t w = r.le4(pos + i) & keep;
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
                const uint32_t rem = n - i;
                const uint32_t keep = rem >= 4 ? 0xFFFFFFFFu : (1u << (8 * rem)) - 1u;
                eq = t[i >> 2] == (r.le4(pos + i) & keep);
            }
            if (eq) return e.id;
        }
    }
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
            const uint32_t p = T.index[off + i];
            if (rule_matches(T.rules[rs.rule_first + p], q)) return p;
        }
        return kInf;
    } else {
        const uint32_t *dir = T.index + rs.topics_off;
        uint32_t lo = 0, hi = rs.ntopics;
        while (lo < hi) {
            const uint32_t m = (lo + hi) >> 1;
            if (dir[3 * m] < (uint32_t)tid) lo = m + 1; else hi = m;
        }
        if (lo >= rs.ntopics || dir[3 * lo] != (uint32_t)tid) return kInf;
        off = dir[3 * lo + 1];
        cnt = dir[3 * lo + 2];
    }
    for (uint32_t i = 0; i < cnt; i++) {
        const uint32_t p = T.index[off + i];
        if (rule_matches(T.rules[rs.rule_first + p], q)) return p;
    }
    return kInf;
}

// MatchesRule over a decoded request: ntopics topics whose best first-match
// positions' maximum is cmax.  Returns the allowing rule's position or kInf.
__device__ __forceinline__ uint32_t matches_rule(const KafkaTables &T, const DevKafkaRuleset &rs, const ReqInfo &q,
                                                 uint32_t ntopics, uint32_t cmax) {
    uint32_t best = kInf;
    if (ntopics == 0) {
        const int key = (q.kind >= 0 && q.kind < 64) ? q.kind : 64;
        const uint32_t off = T.index[rs.bykey_off + 2 * key], cnt = T.index[rs.bykey_off + 2 * key + 1];
        for (uint32_t i = 0; i < cnt; i++) {
            const uint32_t p = T.index[off + i];
            if (rule_matches(T.rules[rs.rule_first + p], q)) { best = p; break; }
        }
    } else {
        for (uint32_t i = 0; i < rs.ntopicless; i++) {
            const uint32_t p = T.index[rs.topicless_off + i];
            if (p >= cmax) break;  // cannot beat topic completion
            if (rule_matches(T.rules[rs.rule_first + p], q)) { best = p; break; }
        }
        if (best == kInf) best = cmax;
    }
    return best;
}

// ---------------- the exact lane-serial path ----------------
struct ExactHooks {
    const KafkaTables &T;
    const DevKafkaRuleset &rs;
    ReqInfo &q;
    GRd &r;
    const uint8_t *lds;
    uint32_t ntopics, cmax;
    __device__ __forceinline__ void client(uint32_t o, uint32_t l) {
        q.client = str_lookup(T.client_hash, T.client_mask, T.strings, r, o, l);
        if (q.client < 0) q.client = -2;
    }
    __device__ __forceinline__ void topic(uint32_t o, uint32_t l) {
        if (q.typed != 1) return;
        ntopics++;
        const int32_t tid = l > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, r, o, l) : -1;
        const uint32_t e = topic_first(T, rs, q, tid);
        cmax = cmax > e ? cmax : e;
    }
    // CRC32-IEEE of [pos, pos + n), 8 bytes per step from the nibble tables
    __device__ __forceinline__ bool msg(uint32_t pos, uint32_t n, uint32_t stored) {
        uint32_t c = 0xFFFFFFFFu, i = 0;
        for (; i + 8 <= n; i += 8) c = crc_step8n(lds, r.le4(pos + i) ^ c, r.le4(pos + i + 4));
        for (; i < n; i++) c = crc_byte(lds, c, (uint32_t)r.be(pos + i, 1));
        return ~c == stored;
    }
};

// One request through the reference's path (HBM bytes, CRC inline); false if
// the entry is left to another protocol's kernel (no output).
__device__ __noinline__ bool classify_exact(const Batch &B, const KafkaTables &T, const uint8_t *lds, DevConn conn,
                                            uint64_t off, uint32_t len, uint32_t answer_other, uint8_t &verdict,
                                            int32_t &rule, uint32_t &consumed, bool &zflag) {
    verdict = V_PARSE_ERROR;
    rule = -1;
    consumed = 0;
    zflag = false;
    if (conn.proto != PROTO_KAFKA || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
        if (!answer_other || (L7_PROTO_OWNED(conn.proto) && conn.proto != PROTO_KAFKA)) return false;
        verdict = V_UNSUPPORTED;  // unknown connection / no parser
        return true;
    }
    if (!l7_in_arena(off, len, B.arena_len)) { verdict = V_UNSUPPORTED; return true; }  // out of contract
    GRd r{B.arena + off, {}};
    r.cur.line = ~(uintptr_t)0;
    // ---- proto.ReadReq
    if (len < 4) { verdict = V_INCOMPLETE; return true; }
    const int32_t size = (int32_t)r.be(0, 4);
    if (size <= 0) return true;
    if (len < 6) { verdict = V_INCOMPLETE; return true; }
    if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) return true;
    const uint32_t rawlen = (uint32_t)size + 4;
    if (rawlen > len) { verdict = V_INCOMPLETE; return true; }
    if (rawlen < 12) return true;
    ReqInfo q;
    q.kind = (int16_t)r.be(4, 2);
    q.version = (int16_t)r.be(6, 2);
    q.typed = kind_typed(q.kind);
    q.client = -2;
    const DevKafkaRuleset &rs = T.rulesets[conn.ruleset];
    ExactHooks h{T, rs, q, r, lds, 0, 0};
    if (q.typed && kafka_walk(r, rawlen, q.kind, zflag, h) == -1) return true;
    consumed = rawlen;
    verdict = V_DENY;
    if (!rs.any) return true;
    const uint32_t best = matches_rule(T, rs, q, h.ntopics, h.cmax);
    if (best != kInf) { verdict = V_ALLOW; rule = T.rules[rs.rule_first + best].gid; }
    return true;
}

// ---------------- the deferred walk's hooks ----------------
struct DeferHooks {
    uint8_t *lds;
    uint32_t W;    // the wave's LDS region
    uint32_t at;   // the request's byte 0, as an offset in the wave's buffer
    uint32_t lane;
    bool topics_on;
    uint32_t ntopics, co, cl;
    bool redo;
    __device__ __forceinline__ void client(uint32_t o, uint32_t l) { co = o; cl = l; }
    __device__ __forceinline__ void topic(uint32_t o, uint32_t l) {
        if (!topics_on) return;
        ntopics++;
        if (l > 255) { redo = true; return; }
        const uint32_t t = atomicAdd(reinterpret_cast<uint32_t *>(lds + W + W_NT), 1u);
        if (t >= kMaxTopics) { redo = true; return; }
        reinterpret_cast<uint32_t *>(lds + W + W_TR)[t] = (at + o) | l << 14 | lane << 22;
    }
    __device__ __forceinline__ bool msg(uint32_t pos, uint32_t n, uint32_t stored) {
        if (n < 4) { redo = true; return true; }  // the initial register spans past the message
        const uint32_t s = (n + kSeg - 1) / kSeg;
        const uint32_t old = atomicAdd(reinterpret_cast<uint32_t *>(lds + W + W_CTR), (1u << 16) | s);
        const uint32_t k = old >> 16, sp = old & 0xFFFF;
        if (k >= kMaxMsgs) { redo = true; return true; }
        if (sp + s > kMaxSegs) redo = true;  // its tail segments are not hashed: the check fails, the exact path decides
        reinterpret_cast<uint16_t *>(lds + W + W_MA)[k] = (uint16_t)(at + pos);
        reinterpret_cast<uint16_t *>(lds + W + W_ML)[k] = (uint16_t)n;
        reinterpret_cast<uint16_t *>(lds + W + W_MS)[k] = (uint16_t)sp;
        (lds + W + W_MO)[k] = (uint8_t)lane;
        reinterpret_cast<uint32_t *>(lds + W + W_MC)[k] = stored;
        reinterpret_cast<uint32_t *>(lds + W + W_MX)[k] = 0;
        if (sp < kMaxSegs) (lds + W + W_SF)[sp] = (uint8_t)(k + 1);
        return true;
    }
};

// ballot helpers: the nearest flagged lane at or below this one
__device__ __forceinline__ uint64_t upto_mask(uint32_t lane) { return (2ull << lane) - 1ull; }

}  // namespace

// Phase timing (experiment builds with -DL7G_KAFKA_PHASES only): cycles per
// wave in stage / walk / lookups / CRC / verdicts / exact path, then the
// counts of sub-batches and of exact-path lanes.
#ifdef L7G_KAFKA_PHASES
__device__ unsigned long long g_kphase[8];
#define KPH_DECL uint64_t kph[8] = {}; uint64_t kph_t = __builtin_amdgcn_s_memtime();
#define KPH(i) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); kph[i] += t_ - kph_t; kph_t = t_; } while (0)
#define KPH_COUNT(i, v) (kph[i] += (v))
#define KPH_FLUSH() do { if ((threadIdx.x & 63) == 0) for (int i_ = 0; i_ < 8; i_++) atomicAdd(&g_kphase[i_], (unsigned long long)kph[i_]); } while (0)
#else
#define KPH_DECL
#define KPH(i) do {} while (0)
#define KPH_COUNT(i, v) do {} while (0)
#define KPH_FLUSH() do {} while (0)
#endif

// sel: this protocol's request indices from partition_kernel (mixed batches),
// else requests 0..n-1.  answer_other: answer entries on connections that are
// not Kafka (single-protocol engines, where partition_kernel does not run).
__global__ __launch_bounds__(kBlock) void kafka_classify_kernel(Batch B, KafkaTables T, const uint32_t *__restrict__ sel,
                                                                const uint32_t *__restrict__ sel_count,
                                                                uint32_t answer_other, uint32_t *__restrict__ zlist,
                                                                uint32_t *__restrict__ zcount,
                                                                uint32_t *__restrict__ work) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
    const uint32_t n = B.n;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    {
        const uint32_t *src = reinterpret_cast<const uint32_t *>(&kCrcNib);
        for (uint32_t i = threadIdx.x; i < kTabBytes / 4; i += kBlock) reinterpret_cast<uint32_t *>(lds)[i] = src[i];
    }
    __syncthreads();
    const uint32_t W = kTabBytes + wave * kWaveBytes;
    // (L7_KAFKA_CLASSES length classes, class c at sel + c * n, sel_count[c] entries each)
    constexpr int kCls = L7_KAFKA_CLASSES;
    uint32_t kc[kCls] = {n};
    uint32_t m = n;
    if (sel) {
        m = 0;
        for (int c = 0; c < kCls; c++) { kc[c] = sel_count[c]; m += kc[c]; }
    }
    // A wave takes 64 entries at a time: its first group by position, every
    // later one from a per-launch counter (zeroed by the launcher), so the
    // persistent grid's waves finish together; without a counter, a fixed stride.
    const uint32_t stride = gridDim.x * kBlock;
    uint32_t base = (blockIdx.x * kWaves + wave) * 64;
    KPH_DECL
    for (; base < m;) {
        const uint32_t i = base + lane;
        const bool act = i < m;
        uint32_t idx = i;
        if (act && sel) {
            // the length classes longest first: long produce requests start first, short ones fill the tail
            uint32_t c = kCls - 1, j = i;
            while (c > 0 && j >= kc[c]) { j -= kc[c]; c--; }
            idx = sel[(size_t)c * n + j];
        }
        DevConn conn{-1, PROTO_NONE, 0, 0xFFFF};
        uint64_t off = 0;
        uint32_t len = 0;
        if (act) {
            const uint32_t ci = B.conn_ids[idx];
            off = B.offs[idx];
            len = B.lens[idx];
            if (ci < B.nconns) conn = B.conns[ci];
        }
        const bool kafka = act && conn.proto == PROTO_KAFKA && conn.ruleset >= 0 && (uint32_t)conn.ruleset < T.nrulesets;
        const uint64_t A = (uint64_t)(uintptr_t)B.arena + off;  // chunks are 16-byte aligned in the address space
        uint32_t C = 0;
        if (kafka && len > 0 && l7_in_arena(off, len, B.arena_len)) {
            C = (uint32_t)(((A + len + 15) >> 4) - (A >> 4));
            if (C > kCapChunks) C = 0;
        }
        bool exact = act && C == 0;
        // inclusive prefix of the chunk counts, in lane order
        uint32_t pf = C;
#pragma unroll
        for (uint32_t d = 1; d < 64; d <<= 1) {
            const uint32_t y = __shfl_up(pf, d);
            if (lane >= d) pf += y;
        }
        uint64_t left = __ballot(C != 0);
        KPH(4);
        while (left) {
            KPH_COUNT(6, 1);
            // ---- the next sub-batch: the lanes from the first one left whose chunks fit kCap
            const uint32_t first = (uint32_t)__builtin_ctzll(left);
            const uint32_t pbase = (uint32_t)__builtin_amdgcn_readlane((int)pf, (int)first) -
                                   (uint32_t)__builtin_amdgcn_readlane((int)C, (int)first);
            const uint64_t sub = __ballot(((left >> lane) & 1) && pf - pbase <= kCapChunks);
            left &= ~sub;
            const bool in = (sub >> lane) & 1;
            const uint32_t last = 63 - (uint32_t)__builtin_clzll(sub);
            const uint32_t used = (uint32_t)__builtin_amdgcn_readlane((int)pf, (int)last) - pbase;
            const uint32_t P = pf - C - pbase;  // first chunk of this lane's request in the buffer
            // clear the start flags and counters, then flag each request's first chunk
            {
                uint32_t *fw = reinterpret_cast<uint32_t *>(lds + W + W_CF);
                for (uint32_t k = lane; k < (kCapChunks + kMaxSegs) / 4; k += 64) fw[k] = 0;
                if (lane < 4) reinterpret_cast<uint32_t *>(lds + W + W_CTR)[lane] = 0;
                wave_sync();
                if (in) (lds + W + W_CF)[P] = (uint8_t)(lane + 1);
                wave_sync();
            }
            // ---- stage: 64 chunks per LDS-DMA instruction, chunk -> request by the nearest start flag
            {
                const uint64_t srcb = (A & ~15ull) - 16ull * P;
                uint32_t carry = 0;
                for (uint32_t q = 0; q * 64 < used; q++) {
                    const uint32_t g = q * 64 + lane;
                    const uint32_t f = g < used ? (lds + W + W_CF)[g] : 0u;
                    const uint64_t up = __ballot(f != 0) & upto_mask(lane);
                    const uint32_t from = up ? 63 - (uint32_t)__builtin_clzll(up) : 0u;
                    const uint32_t fo = (uint32_t)__shfl((int)f, (int)from);
                    const uint32_t own = up ? fo : carry;
                    carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
                    const uint64_t sb = __shfl((unsigned long long)srcb, (int)(own - 1));
                    if (g < used)
                        __builtin_amdgcn_global_load_lds((const void *)(uintptr_t)(sb + 16ull * g),
                                                         (__attribute__((address_space(3))) void *)(lds + W + W_BUF +
                                                                                                     q * 1024),
                                                         16, 0, 0);
                }
                asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                __builtin_amdgcn_wave_barrier();
            }
            KPH(0);
            // ---- walk: one lane per request, from LDS, CRCs and lookups deferred
            uint8_t verdict = V_PARSE_ERROR;
            int32_t rule = -1;
            uint32_t consumed = 0;
            bool zflag = false, pending = false;  // pending: decoded, MatchesRule to do
            int kind = 0, ver = 0;
            DeferHooks h{lds, W, 16 * P + (uint32_t)(A & 15), lane, false, 0, 0, 0, false};
            if (in) {
                LRd r{lds, W + W_BUF + h.at};
                do {
                    if (len < 4) { verdict = V_INCOMPLETE; break; }
                    const int32_t size = (int32_t)r.be(0, 4);
                    if (size <= 0) break;
                    if (len < 6) { verdict = V_INCOMPLETE; break; }
                    if ((uint64_t)(uint32_t)size + 4 > kMaxParseBuf) break;
                    const uint32_t rawlen = (uint32_t)size + 4;
                    if (rawlen > len) { verdict = V_INCOMPLETE; break; }
                    if (rawlen < 12) break;
                    kind = (int16_t)r.be(4, 2);
                    ver = (int16_t)r.be(6, 2);
                    const int typed = kind_typed(kind);
                    h.topics_on = typed == 1;
                    if (typed && kafka_walk(r, rawlen, kind, zflag, h) == -1) break;
                    consumed = rawlen;
                    pending = true;
                } while (false);
                reinterpret_cast<int32_t *>(lds + W + W_LR)[lane] = conn.ruleset;
                reinterpret_cast<uint32_t *>(lds + W + W_LQ)[lane] = ((uint32_t)kind & 0xFFFF) | (uint32_t)ver << 16;
                reinterpret_cast<uint32_t *>(lds + W + W_LM)[lane] = 0;
            }
            wave_sync();
            KPH(1);
            // ---- lookups: client ids (a lane per request), then topics (a lane per topic)
            {
                int32_t client = -2;
                if (in && pending && h.cl > 0) {
                    LRd r{lds, W + W_BUF};
                    client = str_lookup(T.client_hash, T.client_mask, T.strings, r, h.at + h.co, h.cl);
                    if (client < 0) client = -2;
                }
                if (in) reinterpret_cast<int32_t *>(lds + W + W_LC)[lane] = client;
                wave_sync();
                uint32_t nt = reinterpret_cast<const uint32_t *>(lds + W + W_NT)[0];
                nt = nt < kMaxTopics ? nt : kMaxTopics;
                for (uint32_t t = lane; t < nt; t += 64) {
                    const uint32_t rec = reinterpret_cast<const uint32_t *>(lds + W + W_TR)[t];
                    const uint32_t o = rec >> 22, tl = (rec >> 14) & 0xFF, tp = rec & 0x3FFF;
                    ReqInfo q;
                    const uint32_t qw = reinterpret_cast<const uint32_t *>(lds + W + W_LQ)[o];
                    q.kind = (int16_t)(qw & 0xFFFF);
                    q.version = (int16_t)(qw >> 16);
                    q.typed = 1;
                    q.client = reinterpret_cast<const int32_t *>(lds + W + W_LC)[o];
                    const DevKafkaRuleset &rs = T.rulesets[reinterpret_cast<const int32_t *>(lds + W + W_LR)[o]];
                    LRd r{lds, W + W_BUF};
                    const int32_t tid = tl > 0 ? str_lookup(T.topic_hash, T.topic_mask, T.strings, r, tp, tl) : -1;
                    const uint32_t e = topic_first(T, rs, q, tid);
                    atomicMax(reinterpret_cast<uint32_t *>(lds + W + W_LM) + o, e);
                }
            }
            wave_sync();
            KPH(2);
            // ---- CRC: a lane per 36-byte segment of the recorded messages
            {
                const uint32_t ctr = reinterpret_cast<const uint32_t *>(lds + W + W_CTR)[0];
                const uint32_t nmsg = (ctr >> 16) < kMaxMsgs ? (ctr >> 16) : kMaxMsgs;
                const uint32_t nseg = (ctr & 0xFFFF) < kMaxSegs ? (ctr & 0xFFFF) : kMaxSegs;
                uint32_t carry = 0;
                for (uint32_t g0 = 0; g0 < nseg; g0 += 64) {
                    const uint32_t g = g0 + lane;
                    const uint32_t f = g < nseg ? (lds + W + W_SF)[g] : 0u;
                    const uint64_t up = __ballot(f != 0) & upto_mask(lane);
                    const uint32_t from = up ? 63 - (uint32_t)__builtin_clzll(up) : 0u;
                    const uint32_t fo = (uint32_t)__shfl((int)f, (int)from);
                    const uint32_t own = up ? fo : carry;  // message + 1
                    carry = (uint32_t)__builtin_amdgcn_readlane((int)own, 63);
                    if (g < nseg && own > 0) {
                        const uint32_t k = own - 1;
                        const uint32_t a = reinterpret_cast<const uint16_t *>(lds + W + W_MA)[k];
                        const uint32_t mlen = reinterpret_cast<const uint16_t *>(lds + W + W_ML)[k];
                        const uint32_t sp = reinterpret_cast<const uint16_t *>(lds + W + W_MS)[k];
                        const uint32_t s = (mlen + kSeg - 1) / kSeg, j = g - sp;
                        if (j < s) {
                            const uint32_t r = mlen - kSeg * (s - 1);  // bytes of the first (partial) segment
                            const int32_t p0 = (int32_t)(r + kSeg * j) - kSeg;  // message position of window byte 0
                            const uint32_t ws = (uint32_t)((int32_t)(W + W_BUF + a) + p0);  // window start (LDS)
                            const uint32_t *wp = reinterpret_cast<const uint32_t *>(lds + (ws & ~3u));
                            uint32_t w[10];
#pragma unroll
                            for (int t = 0; t < 10; t++) w[t] = wp[t];
                            uint32_t x[9];
#pragma unroll
                            for (int t = 0; t < 9; t++) x[t] = __builtin_amdgcn_alignbyte(w[t + 1], w[t], ws & 3);
                            if (p0 < 4) {
                                // bytes before the message are zero; its first four bytes carry the initial register
#pragma unroll
                                for (int t = 0; t < 9; t++) {
                                    const int32_t qq = p0 + 4 * t;
                                    if (qq < 4) {
                                        const uint32_t keep = qq <= -4 ? 0u : qq >= 0 ? ~0u : (~0u << (8 * -qq));
                                        const int32_t low = 4 - qq;
                                        const uint32_t xm = low >= 4 ? ~0u : ((1u << (8 * low)) - 1u);
                                        x[t] = (x[t] & keep) ^ (xm & keep);
                                    }
                                }
                            }
                            uint32_t v = seg_raw(lds, x);
                            uint32_t tsh = s - 1 - j;
                            for (uint32_t b = 0; tsh; b++, tsh >>= 1)
                                if (tsh & 1) v = crc_shift(lds, b, v);
                            atomicXor(reinterpret_cast<uint32_t *>(lds + W + W_MX) + k, v);
                        }
                    }
                }
                wave_sync();
                for (uint32_t k = lane; k < nmsg; k += 64) {
                    const uint32_t acc = reinterpret_cast<const uint32_t *>(lds + W + W_MX)[k];
                    const uint32_t want = reinterpret_cast<const uint32_t *>(lds + W + W_MC)[k];
                    if (~acc != want) {
                        const uint32_t o = (lds + W + W_MO)[k];
                        atomicOr(reinterpret_cast<uint32_t *>(lds + W + W_BAD) + (o >> 5), 1u << (o & 31));
                    }
                }
                wave_sync();
            }
            KPH(3);
            // ---- verdicts
            if (in) {
                const bool crc_bad = (reinterpret_cast<const uint32_t *>(lds + W + W_BAD)[lane >> 5] >> (lane & 31)) & 1;
                if (crc_bad || h.redo) {
                    exact = true;  // the exact path decides it below
                } else {
                    if (pending) {
                        verdict = V_DENY;
                        const DevKafkaRuleset &rs = T.rulesets[conn.ruleset];
                        if (rs.any) {
                            ReqInfo q;
                            q.kind = kind;
                            q.version = ver;
                            q.typed = kind_typed(kind);
                            q.client = reinterpret_cast<const int32_t *>(lds + W + W_LC)[lane];
                            const uint32_t cmax = reinterpret_cast<const uint32_t *>(lds + W + W_LM)[lane];
                            const uint32_t best = matches_rule(T, rs, q, h.ntopics, cmax);
                            if (best != kInf) { verdict = V_ALLOW; rule = T.rules[rs.rule_first + best].gid; }
                        }
                    }
                    B.verdict[idx] = verdict;
                    B.rule[idx] = rule;
                    B.consumed[idx] = consumed;
                    if (zflag && zlist && (verdict == V_ALLOW || verdict == V_DENY)) zlist[atomicAdd(zcount, 1u)] = idx;
                }
            }
            wave_sync();  // the buffer and lists are reused by the next sub-batch
            KPH(4);
        }
        // ---- the exact path: requests over the buffer, CRC failures, list overflows, non-Kafka entries
        KPH_COUNT(7, __popcll(__ballot(exact)));
        if (exact) {
            uint8_t verdict;
            int32_t rule;
            uint32_t consumed;
            bool zflag;
            if (classify_exact(B, T, lds, conn, off, len, answer_other, verdict, rule, consumed, zflag)) {
                B.verdict[idx] = verdict;
                B.rule[idx] = rule;
                B.consumed[idx] = consumed;
                if (zflag && zlist && (verdict == V_ALLOW || verdict == V_DENY)) zlist[atomicAdd(zcount, 1u)] = idx;
            }
        }
        KPH(5);
        // next group
        if (work) {
            uint32_t t = 0;
            if (lane == 0) t = atomicAdd(work, 64u);
            base = stride + (uint32_t)__builtin_amdgcn_readfirstlane((int)t);
        } else {
            base += stride;
        }
    }
    KPH_FLUSH();
}

hipError_t KafkaPhaseTimes(uint64_t *out, bool reset) {
#ifdef L7G_KAFKA_PHASES
    hipError_t rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_kphase), sizeof(uint64_t) * 8);
    if (rc == hipSuccess && reset) {
        const uint64_t z[8] = {};
        rc = hipMemcpyToSymbol(HIP_SYMBOL(g_kphase), z, sizeof z);
    }
    return rc;
#else
    (void)out;
    (void)reset;
    return hipErrorNotSupported;
#endif
}

hipError_t LaunchKafkaClassify(const Batch &B, const KafkaTables &T, const uint32_t *sel, const uint32_t *sel_count,
                               bool answer_other, uint32_t *zlist, uint32_t *zcount, uint32_t *work,
                               hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
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
            resident = 8192;
    }
    if (blocks > (uint32_t)resident) blocks = (uint32_t)resident;
    hipLaunchKernelGGL(kafka_classify_kernel, dim3(blocks), dim3(kBlock), 0, stream, B, T, sel, sel_count,
                       answer_other ? 1u : 0u, zlist, zcount, work);
    return hipGetLastError();
}

}  // namespace l7
