// Device framing of connection streams (product code, l7g_frame_streams /
// l7g_classify_streams in include/l7gpu.h): SURVEY §8 K2 (the Kafka request's
// big-endian int32 size prefix, optiopay proto.ReadReq
// vendor/github.com/optiopay/kafka/proto/messages.go:124-165), P4 (memcached
// text: the command line to "\r\n" plus a storage command's data block,
// proxylib/memcached/text/parser.go:72-262; binary: the 24-byte header plus
// its total body length, binary/parser.go:72-139) and H6 (HTTP/1: the head to
// "\r\n\r\n" plus Content-Length), with r2d2's lines
// (proxylib/r2d2/r2d2parser.go:140-214) and cassandra's 9-byte header plus
// body length (proxylib/cassandra/cassandraparser.go:171-230).
//
// One lane per stream walks it frame by frame and writes each frame's start
// and the bytes from there to the stream's end (the length a parser is handed,
// as proxylib hands OnData's joined input): the classifiers then answer each
// frame, and their consumed length confirms the walk.  The walk stops where a
// frame is incomplete or its length cannot be read ahead of parsing it (a
// chunked HTTP body, a malformed size, a memcached storage line without a byte
// count): that frame is emitted with the rest of the stream, and the caller
// frames what follows after the verdict, as the proxylib op loop does.  These
// are the proposals csrc/proxylib/shim.cc scans on the host (Next*), made on
// the device for many streams at once.
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "gmem.h"

namespace l7 {

namespace {

constexpr int kBlock = 128;

struct Stream {
    const uint8_t *b;  // stream start
    uint64_t n;        // stream bytes
    uint64_t blk;      // the 16-byte block held in w (~0: none)
    uint4 w;
};

// byte i of the stream, through a one-block cache: a lane scanning a line
// issues one 16-byte load per block instead of one (dependent) load per byte
__device__ __forceinline__ uint32_t sbyte(Stream &S, uint64_t i) {
    const uint64_t a = (uint64_t)S.b + i, base = a & ~15ull;
    if (base != S.blk) {
        S.w = gload16(base);
        S.blk = base;
    }
    const uint32_t k = (uint32_t)(a & 15);
    const uint32_t d = k < 8 ? (k < 4 ? S.w.x : S.w.y) : (k < 12 ? S.w.z : S.w.w);
    return (d >> (8 * (k & 3))) & 0xFF;
}

// byte i straight from memory (short lines: the memcached token scan, where
// the block cache's compare and select cost more than the L1 hit they save)
__device__ __forceinline__ uint32_t dbyte(const Stream &S, uint64_t i) { return S.b[i]; }

__device__ __forceinline__ uint32_t eq16(uint4 w, uint32_t c) {  // bit k: byte k of w == c
    const uint32_t cc = c * 0x01010101u;
    auto e = [cc](uint32_t x) {
        const uint32_t t = x ^ cc;
        return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    };
    auto nib = [](uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); };
    return nib(e(w.x)) | nib(e(w.y)) << 4 | nib(e(w.z)) << 8 | nib(e(w.w)) << 12;
}

// 16-byte loads in flight per step of the CRLF scan (1M HTTP requests in 16k
// streams: 4 -> 7.6 ms, 8 -> 6.9, 16 -> 6.7; memcached text 9.1, 8.6, 8.7)
constexpr int kScan = 8;

// first i in [from, S.n) with b[i] == '\r' and b[i + 1] == '\n' (S.n: none),
// 16 * kScan bytes a step
__device__ uint64_t find_crlf(Stream &S, uint64_t from) {
    if (from >= S.n) return S.n;
    const uint64_t a = (uint64_t)S.b + from;
    uint64_t base = a & ~15ull;
    const uint64_t end = (uint64_t)S.b + S.n;
    uint32_t skip = (uint32_t)(a - base);
    uint32_t prev_cr = 0;  // the last block ended in '\r'
    for (; base < end; base += 16 * kScan) {
        uint4 w[kScan];
#pragma unroll
        for (int k = 0; k < kScan; k++)
            if (base + 16 * k < end) w[k] = gload16(base + 16 * k);
#pragma unroll
        for (int k = 0; k < kScan; k++) {
            const uint64_t bk = base + 16 * k;
            if (bk >= end) break;
            uint32_t valid = end - bk >= 16 ? 0xFFFFu : (1u << (uint32_t)(end - bk)) - 1u;
            valid &= 0xFFFFu << skip;
            skip = 0;
            const uint32_t cr = eq16(w[k], '\r') & valid, lf = eq16(w[k], '\n') & valid;
            const uint32_t hit = ((cr << 1) | prev_cr) & lf;  // LF right after a CR
            if (hit) return bk - (uint64_t)S.b + __builtin_ctz(hit) - 1;
            prev_cr = (cr >> 15) & 1;
        }
    }
    return S.n;
}

// NextKafka: [size int32 BE][size bytes]; size <= 0 or past the stream: stop
__device__ uint64_t next_kafka(Stream &S, uint64_t p) {
    if (S.n - p < 4) return 0;
    const int32_t size = (int32_t)(sbyte(S, p) << 24 | sbyte(S, p + 1) << 16 | sbyte(S, p + 2) << 8 | sbyte(S, p + 3));
    if (size <= 0 || (uint64_t)size + 4 > S.n - p) return 0;
    return p + 4 + (uint64_t)size;
}

// NextMcBinary: 24-byte header, total body length at bytes 8..11
__device__ uint64_t next_mc_binary(Stream &S, uint64_t p) {
    if (S.n - p < 24) return 0;
    const uint64_t body = sbyte(S, p + 8) << 24 | sbyte(S, p + 9) << 16 | sbyte(S, p + 10) << 8 | sbyte(S, p + 11);
    return body + 24 <= S.n - p ? p + 24 + body : 0;
}

// bytes.Fields' separators (unicode.IsSpace) at s[i], as shim.cc SpaceLen:
// the width of the space rune there, 0 for none
__device__ uint32_t space_len(Stream &S, uint64_t i, uint64_t n) {
    const uint32_t c = dbyte(S, i);
    if (c == ' ' || (c >= 0x09 && c <= 0x0D)) return 1;
    if (c < 0xC2 || c > 0xE3 || i + 1 >= n) return 0;
    const uint32_t c1 = dbyte(S, i + 1);
    if (c == 0xC2) return (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
    if (i + 2 >= n) return 0;
    const uint32_t c2 = dbyte(S, i + 2);
    if (c == 0xE1) return (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
    if (c == 0xE2 && c1 == 0x80) return ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
    if (c == 0xE2 && c1 == 0x81) return c2 == 0x9F ? 3 : 0;
    if (c == 0xE3) return (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
    return 0;
}

// NextMcText: the line to "\r\n"; set / add / replace / append / prepend / cas
// also carry <bytes> + "\r\n" of data (tokens[4], a non-negative decimal)
__device__ uint64_t next_mc_text(Stream &S, uint64_t p) {
    const uint64_t lf = find_crlf(S, p);
    if (lf >= S.n) return 0;
    // tokens 0 and 4 of the line [p, lf)
    uint64_t t0 = 0, t0e = 0, t4 = 0, t4e = 0;
    uint32_t nt = 0;
    bool in = false;
    for (uint64_t i = p; i < lf;) {
        const uint32_t sp = space_len(S, i, lf);
        if (sp) {
            if (in) {
                if (nt == 0) t0e = i;
                if (nt == 4) t4e = i;
                nt++;
            }
            in = false;
            i += sp;
        } else {
            if (!in) {
                if (nt == 0) t0 = i;
                if (nt == 4) t4 = i;
                in = true;
            }
            i++;
        }
        if (nt > 4) break;
    }
    if (in) {
        if (nt == 0) t0e = lf;
        if (nt == 4) t4e = lf;
        nt++;
    }
    uint64_t next = lf + 2;
    bool storage = false;
    if (nt >= 1) {
        const uint64_t k = t0e - t0;
        auto is = [&](const char *w, uint64_t wl) {
            if (k != wl) return false;
            for (uint64_t j = 0; j < wl; j++)
                if (dbyte(S, t0 + j) != (uint32_t)(uint8_t)w[j]) return false;
            return true;
        };
        storage = is("set", 3) || is("add", 3) || is("replace", 7) || is("append", 6) || is("prepend", 7) || is("cas", 3);
    }
    if (storage) {
        if (nt < 5) return 0;
        // strtoll(tokens[4]) with the whole token consumed, >= 0
        uint64_t i = t4;
        bool neg = false;
        if (i < t4e && (dbyte(S, i) == '+' || dbyte(S, i) == '-')) {
            neg = dbyte(S, i) == '-';
            i++;
        }
        if (i >= t4e) return 0;
        uint64_t v = 0;
        for (; i < t4e; i++) {
            const uint32_t d = dbyte(S, i) - '0';
            if (d > 9) return 0;
            v = v * 10 + d;
            if (v > (1ull << 40)) return 0;  // (strtoll saturates; no such frame fits a stream)
        }
        if (neg && v) return 0;
        next += v + 2;
    }
    return next <= S.n ? next : 0;
}

// NextLine (r2d2): to "\r\n"
__device__ uint64_t next_line(Stream &S, uint64_t p) {
    const uint64_t lf = find_crlf(S, p);
    return lf >= S.n ? 0 : lf + 2;
}

__device__ __forceinline__ uint32_t lower(uint32_t c) { return c - 'A' < 26u ? c + 32 : c; }

// NextHttp: the head to "\r\n\r\n" plus Content-Length (strtoull of the value);
// a Transfer-Encoding header stops the walk (chunked bodies are framed by the
// classifier)
__device__ uint64_t next_http(Stream &S, uint64_t p) {
    uint64_t ls = find_crlf(S, p);
    if (ls >= S.n) return 0;
    ls += 2;
    uint64_t cl = 0;
    for (;;) {  // header lines until the empty one
        const uint64_t le = find_crlf(S, ls);
        if (le >= S.n) return 0;  // no "\r\n\r\n": incomplete
        if (le == ls) break;      // the empty line: the head ends at ls + 2
        // the name is the line up to its first ':'; the two names that matter
        // hold no ':', so a line names one iff its ':' sits right after it
        // (no byte-wise colon scan of every header line)
        auto name_is = [&](const char *w, uint64_t wl) {
            if (le - ls <= wl || sbyte(S, ls + wl) != ':') return false;
            for (uint64_t j = 0; j < wl; j++)
                if (lower(sbyte(S, ls + j)) != (uint32_t)(uint8_t)w[j]) return false;
            return true;
        };
        if (name_is("transfer-encoding", 17)) return 0;
        if (name_is("content-length", 14)) {  // strtoull: leading spaces, optional sign, digits
            uint64_t i = ls + 15;
            while (i < S.n && (sbyte(S, i) == ' ' || (sbyte(S, i) >= 0x09 && sbyte(S, i) <= 0x0D))) i++;
            bool neg = false;
            if (i < S.n && (sbyte(S, i) == '+' || sbyte(S, i) == '-')) {
                neg = sbyte(S, i) == '-';
                i++;
            }
            uint64_t v = 0;
            bool over = false;
            for (; i < S.n; i++) {
                const uint32_t d = sbyte(S, i) - '0';
                if (d > 9) break;
                if (v > (~0ull - d) / 10) over = true;
                v = over ? ~0ull : v * 10 + d;
            }
            cl = neg ? 0 - v : v;
        }
        ls = le + 2;
    }
    const uint64_t head_end = ls + 2;
    if (cl > S.n - head_end) return 0;
    return head_end + cl;
}

// cassandra: 9-byte header, body length at bytes 5..8
__device__ uint64_t next_cassandra(Stream &S, uint64_t p) {
    if (S.n - p < 9) return 0;
    const uint64_t fl = 9 + (uint64_t)(sbyte(S, p + 5) << 24 | sbyte(S, p + 6) << 16 | sbyte(S, p + 7) << 8 | sbyte(S, p + 8));
    return fl <= S.n - p ? p + fl : 0;
}


// ---------------- text streams (HTTP, memcached text, r2d2): a wave per stream ----------------
// A window is 1 KiB of the stream's address range, 16-byte aligned: lane l
// holds chunk l in registers with its "\r\n" mask (bit k: byte k is '\r' and
// the byte after it '\n') and, for memcached text, its separator mask (bit k:
// byte k belongs to a unicode.IsSpace rune as bytes.Fields reads them).  One
// load instruction brings the whole window (64 lanes x 16 bytes, coalesced);
// the CR/LF search is a ballot over the lanes' masks.  The frame walk itself
// is wave-uniform scalar code that reads those registers with v_readlane, so
// the wave does the work the one-lane walk did, 64 bytes at a time.
constexpr uint32_t kWinBytes = 1024;

// Phase timing (experiment builds with -DL7G_FRAME_PHASES only): per wave, the
// cycles in window loads (the load and the masks), the cycles of whole
// streams, the window loads and the frames.
#ifdef L7G_FRAME_PHASES
__device__ unsigned long long g_fphase[8];
#define FPH(x) x
#else
#define FPH(x)
#endif

struct TWin {
    const uint8_t *A;  // stream start
    uint64_t n;        // stream bytes
    uint64_t wa;       // the window's address (16-byte aligned); ~0: none
    uint64_t ends;     // lanes whose chunk holds a CRLF start
    uint4 w;           // this lane's chunk
    uint32_t crlf, sp; // this lane's masks
    bool want_sp;
    // HTTP (want_http): bit k of dcrlf: "\r\n\r\n" starts at byte k; of te / cl:
    // a line starts at byte k (right after a CRLF) naming transfer-encoding /
    // content-length; te_any / cl_any / dc_any: the lanes with any
    bool want_http;
    uint32_t dcrlf, te, cl;
    uint64_t te_any, cl_any, dc_any;
    // the window after this one's vouched-for part (HTTP scans move on to it),
    // fetched while this one is scanned
    uint64_t nwa;
    uint4 nw;
    FPH(uint64_t ph_load; uint64_t ph_n;)
};

__device__ __forceinline__ uint32_t rl(uint32_t v, uint32_t l) { return (uint32_t)__builtin_amdgcn_readlane((int)v, (int)l); }

__device__ __forceinline__ void twin_masks(TWin &W) {
    const uint32_t lane = threadIdx.x & 63;
    const uint64_t s0 = (uint64_t)W.A, s1 = s0 + W.n;
    const uint64_t ca = W.wa + 16ull * lane;
    uint32_t vm = 0;  // bytes of this chunk inside the stream
    if (ca + 16 > s0 && ca < s1) {
        const uint32_t lo = ca >= s0 ? 0u : (uint32_t)(s0 - ca);
        const uint32_t hi = ca + 16 <= s1 ? 16u : (uint32_t)(s1 - ca);
        vm = (0xFFFFu << lo) & (0xFFFFu >> (16 - hi));
    }
    const uint4 w = W.w;
    const uint32_t cr = eq16(w, '\r') & vm, lf = eq16(w, '\n') & vm;
    uint32_t nlf = (uint32_t)__shfl_down((int)lf, 1) & 1u;  // the next chunk's first byte is '\n'
    if (lane == 63) nlf = 0;                                 // (past the window: the next window decides)
    W.crlf = cr & ((lf >> 1) | (nlf << 15));
    W.ends = __ballot(W.crlf != 0);
    if (W.want_http) {
        // "\r\n\r\n": a CRLF two bytes after a CRLF (the next chunk's first two bits from lane + 1)
        uint32_t ncr = (uint32_t)__shfl_down((int)W.crlf, 1) & 3u;
        if (lane == 63) ncr = 0;
        W.dcrlf = W.crlf & ((W.crlf >> 2) | (ncr << 14));
        // line starts: two bytes after a CRLF (bits 14, 15 of the previous chunk's carry over)
        const uint32_t pcr = (uint32_t)__shfl_up((int)W.crlf, 1);
        const uint32_t starts = ((W.crlf << 2) | (lane ? (pcr >> 14) & 3u : 0u)) & 0xFFFFu;
        // only a line starting with c / C / t / T can name either: the 18 bytes
        // from such a start (this chunk and the next two lanes') are read only
        // when some lane has one
        const uint32_t cand = starts & (eq16(w, 'c') | eq16(w, 'C') | eq16(w, 't') | eq16(w, 'T'));
        uint32_t te = 0, clm = 0;
        if (__ballot(cand != 0)) {
            uint32_t x[12];
            x[0] = w.x; x[1] = w.y; x[2] = w.z; x[3] = w.w;
            x[4] = (uint32_t)__shfl_down((int)w.x, 1); x[5] = (uint32_t)__shfl_down((int)w.y, 1);
            x[6] = (uint32_t)__shfl_down((int)w.z, 1); x[7] = (uint32_t)__shfl_down((int)w.w, 1);
            x[8] = (uint32_t)__shfl_down((int)w.x, 2); x[9] = (uint32_t)__shfl_down((int)w.y, 2);
            x[10] = (uint32_t)__shfl_down((int)w.z, 2); x[11] = (uint32_t)__shfl_down((int)w.w, 2);
            for (uint32_t sm = cand; sm; sm &= sm - 1) {
                const uint32_t k = __builtin_ctz(sm), q = k >> 2, sh = k & 3;
                uint32_t a[5];
#pragma unroll
                for (int i = 0; i < 5; i++) {
                    const uint32_t lo = q == 0 ? x[i] : q == 1 ? x[i + 1] : q == 2 ? x[i + 2] : x[i + 3];
                    const uint32_t hi = q == 0 ? x[i + 1] : q == 1 ? x[i + 2] : q == 2 ? x[i + 3] : x[i + 4];
                    a[i] = __builtin_amdgcn_alignbyte(hi, lo, sh);
                }
                // content-length: "cont" "ent-" "leng" "th" ':' (letters lower-cased, '-' and ':' exact)
                if ((a[0] | 0x20202020u) == 0x746e6f63u && (a[1] | 0x00202020u) == 0x2d746e65u &&
                    (a[2] | 0x20202020u) == 0x676e656cu && ((a[3] | 0x00002020u) & 0x00FFFFFFu) == 0x003a6874u)
                    clm |= 1u << k;
                // transfer-encoding: "tran" "sfer" "-enc" "odin" "g:"
                if ((a[0] | 0x20202020u) == 0x6e617274u && (a[1] | 0x20202020u) == 0x72656673u &&
                    (a[2] | 0x20202000u) == 0x636e652du && (a[3] | 0x20202020u) == 0x6e69646fu &&
                    ((a[4] | 0x00000020u) & 0xFFFFu) == 0x3a67u)
                    te |= 1u << k;
            }
        }
        W.te = te;
        W.cl = clm;
        W.te_any = __ballot(te != 0);
        W.cl_any = __ballot(clm != 0);
        W.dc_any = __ballot(W.dcrlf != 0);
    }
    if (W.want_sp) {
        // separators of bytes.Fields (shim.cc SpaceLen): ASCII White_Space by
        // SWAR compares, and the multi-byte runes from their lead bytes (0xC2,
        // 0xE1-0xE3: never a continuation byte, so a rune start is judged on its
        // own bytes; its end lies before any CR), byte by byte only where a lead
        // byte is
        const uint32_t asc = eq16(w, 0x20) | eq16(w, 0x09) | eq16(w, 0x0A) | eq16(w, 0x0B) | eq16(w, 0x0C) |
                             eq16(w, 0x0D);
        const uint32_t lead = eq16(w, 0xC2) | eq16(w, 0xE1) | eq16(w, 0xE2) | eq16(w, 0xE3);
        const uint32_t nx = (uint32_t)__shfl_down((int)w.x, 1);
        const uint32_t nxt = lane == 63 ? 0u : nx & 0xFFFFu;  // the next chunk's first two bytes
        uint32_t s2 = 0, s3 = 0;
        for (uint32_t lm = lead; lm; lm &= lm - 1) {
            const int k = __builtin_ctz(lm);
            auto at = [&](int q) -> uint32_t {  // byte q of the chunk, past 15 from the next one
                if (q < 16) {
                    const uint32_t wq = q < 4 ? w.x : q < 8 ? w.y : q < 12 ? w.z : w.w;
                    return (wq >> (8 * (q & 3))) & 0xFF;
                }
                return (nxt >> (8 * (q - 16))) & 0xFF;
            };
            const uint32_t b = at(k), b1 = at(k + 1), b2 = at(k + 2);
            if (b == 0xC2 && (b1 == 0x85 || b1 == 0xA0)) s2 |= 1u << k;
            const bool r3 = (b == 0xE1 && b1 == 0x9A && b2 == 0x80) ||
                            (b == 0xE2 && b1 == 0x80 && ((b2 >= 0x80 && b2 <= 0x8A) || b2 == 0xA8 || b2 == 0xA9 || b2 == 0xAF)) ||
                            (b == 0xE2 && b1 == 0x81 && b2 == 0x9F) || (b == 0xE3 && b1 == 0x80 && b2 == 0x80);
            if (r3) s3 |= 1u << k;
        }
        // a rune started in the previous chunk's last bytes covers this one's first
        const uint32_t ps2 = (uint32_t)__shfl_up((int)s2, 1), ps3 = (uint32_t)__shfl_up((int)s3, 1);
        const uint32_t carry = lane == 0 ? 0u : ((ps2 >> 15) & 1) | ((ps3 >> 14) & 1) | (((ps3 >> 15) & 1) * 3u);
        W.sp = (asc | s2 | (s2 << 1) | s3 | (s3 << 1) | (s3 << 2) | carry) & 0xFFFFu;
    }
}
// this lane's chunk of the window at wa (zero outside the stream)
__device__ __forceinline__ uint4 twin_chunk(const TWin &W, uint64_t wa) {
    const uint64_t ca = wa + 16ull * (threadIdx.x & 63);
    uint4 w = make_uint4(0, 0, 0, 0);
    if (ca + 16 > (uint64_t)W.A && ca < (uint64_t)W.A + W.n) w = gload16(ca);
    return w;
}
// An HTTP scan trusts a window's first kHttpSure bytes (the masks of its last
// two chunks need bytes past it) and goes on in a window one chunk before that
// point, so that a header line starting at the first bytes it has not trusted
// has the CRLF before it (and its line-start bit) inside the new window.
constexpr uint32_t kHttpSure = kWinBytes - 32;
constexpr uint32_t kNextWin = kHttpSure - 16;  // where an HTTP scan's next window starts
// load the window at address wa
__device__ __forceinline__ void twin_load(TWin &W, uint64_t wa) {
    FPH(const uint64_t t0_ = __builtin_amdgcn_s_memtime();)
    W.w = W.want_http && wa == W.nwa ? W.nw : twin_chunk(W, wa);
    W.wa = wa;
    if (W.want_http) {  // the next one, in flight while this one is scanned
        W.nwa = wa + kNextWin < (uint64_t)W.A + W.n ? wa + kNextWin : ~0ull;
        if (W.nwa != ~0ull) W.nw = twin_chunk(W, W.nwa);
    }
    twin_masks(W);
    FPH(W.ph_load += __builtin_amdgcn_s_memtime() - t0_; W.ph_n++;)
}
// a window holding stream offset x and the need - 1 bytes after it
__device__ __forceinline__ void twin_at(TWin &W, uint64_t x, uint32_t need = 1) {
    const uint64_t a = (uint64_t)W.A + x;
    if (W.wa == ~0ull || a < W.wa || a + need > W.wa + kWinBytes) twin_load(W, a & ~15ull);
}
// stream byte x (x < n)
__device__ __forceinline__ uint32_t tbyte(TWin &W, uint64_t x) {
    twin_at(W, x);
    const uint32_t r = (uint32_t)((uint64_t)W.A + x - W.wa), c = r >> 4, k = r & 15;
    const uint32_t d = k < 4 ? rl(W.w.x, c) : k < 8 ? rl(W.w.y, c) : k < 12 ? rl(W.w.z, c) : rl(W.w.w, c);
    return (d >> (8 * (k & 3))) & 0xFF;
}
// first i in [from, n) with b[i] == '\r' and b[i + 1] == '\n' (n: none), a
// window at a time; consecutive windows overlap by one chunk, so a CRLF split by
// a window's end is judged in the next one
__device__ __forceinline__ uint64_t tfind_crlf(TWin &W, uint64_t from) {
    if (from >= W.n) return W.n;
    twin_at(W, from, 32);
    for (;;) {
        const uint32_t r = (uint32_t)((uint64_t)W.A + from - W.wa);
        const uint32_t c = r >> 4;
        const uint32_t m0 = rl(W.crlf, c) & (0xFFFFu << (r & 15));
        if (m0) return W.wa + 16ull * c + __builtin_ctz(m0) - (uint64_t)W.A;
        const uint64_t rest = c >= 63 ? 0ull : W.ends & (~0ull << (c + 1));
        if (rest) {
            const uint32_t c2 = (uint32_t)__builtin_ctzll(rest);
            return W.wa + 16ull * c2 + __builtin_ctz(rl(W.crlf, c2)) - (uint64_t)W.A;
        }
        if (W.wa + kWinBytes >= (uint64_t)W.A + W.n) return W.n;  // the window reaches the stream's end
        // on to the next window (it overlaps this one by a chunk: a CRLF cut by
        // this one's end is judged there)
        const uint64_t nw = W.wa + kWinBytes - 16;
        from = nw - (uint64_t)W.A > from ? nw - (uint64_t)W.A : from;
        twin_load(W, nw);
    }
}
// 4 stream bytes at x, little-endian (bytes past n are 0)
__device__ __forceinline__ uint32_t tword(TWin &W, uint64_t x) {
    twin_at(W, x, 4);
    const uint32_t r = (uint32_t)((uint64_t)W.A + x - W.wa);
    const uint32_t i = r >> 2;
    const uint32_t lo_c = i >> 2, lo_j = i & 3, hi_i = i + 1, hi_c = hi_i >> 2, hi_j = hi_i & 3;
    auto word = [&](uint32_t c, uint32_t j) {
        return j == 0 ? rl(W.w.x, c) : j == 1 ? rl(W.w.y, c) : j == 2 ? rl(W.w.z, c) : rl(W.w.w, c);
    };
    const uint32_t lo = word(lo_c, lo_j), hi = hi_c < 64 ? word(hi_c, hi_j) : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, r & 3);
}

// NextHttp on the window (next_http's semantics).  The request line ends at
// the first CRLF; the head ends at the first "\r\n\r\n" from there (the
// line-by-line walk's first empty line); a transfer-encoding line start in
// between stops the walk, and the last content-length line start gives the
// body length.  The masks of a window's last 32 bytes need bytes past it, so a
// window vouches for its first 992 bytes (all of them when it holds the
// stream's end) and the scan goes on from there in the window that starts one
// chunk earlier (kNextWin): lane 0's line starts take no carry from a previous
// chunk, so a line starting at byte 992 or 993 is seen only with the CRLF
// before it in the same window.
// bits of lanes [c0, c1] (c0 <= c1 < 64)
__device__ __forceinline__ uint64_t lanes_between(uint32_t c0, uint32_t c1) {
    const uint64_t hi = c1 >= 63 ? ~0ull : (2ull << c1) - 1;
    return hi & (~0ull << c0);
}
__device__ __forceinline__ uint64_t tnext_http(TWin &W, uint64_t p) {
    const uint64_t rle = tfind_crlf(W, p);  // the request line's CRLF
    if (rle >= W.n) return 0;
    uint64_t x = rle;         // scan position (stream offset)
    uint64_t last_cl = ~0ull; // the last content-length line start
    uint64_t e = ~0ull;       // the "\r\n\r\n"
    for (;;) {
        twin_at(W, x, 64);
        const uint64_t s_end = W.wa + kWinBytes >= (uint64_t)W.A + W.n ? W.wa + kWinBytes : W.wa + kHttpSure;
        const uint32_t r0 = (uint32_t)((uint64_t)W.A + x - W.wa), r1 = (uint32_t)(s_end - W.wa);  // [r0, r1) vouched for
        // the first "\r\n\r\n" at or after r0
        uint32_t re = r1;
        {
            const uint32_t c = r0 >> 4;
            const uint32_t m0 = rl(W.dcrlf, c) & (0xFFFFu << (r0 & 15));
            if (m0) re = 16 * c + __builtin_ctz(m0);
            else {
                const uint64_t rest = c >= 63 ? 0ull : W.dc_any & (~0ull << (c + 1));
                if (rest) {
                    const uint32_t c2 = (uint32_t)__builtin_ctzll(rest);
                    re = 16 * c2 + __builtin_ctz(rl(W.dcrlf, c2));
                }
            }
            if (re > r1) re = r1;
        }
        const bool found = re < r1;
        // header line starts in [r0, re + 2) (the empty line's own start names nothing)
        const uint32_t lim = found ? re + 2 : r1;
        if (lim > r0) {
            const uint32_t c0 = r0 >> 4, c1 = (lim - 1) >> 4;
            const uint64_t span = lanes_between(c0, c1);
            auto in_range = [&](uint32_t m, uint32_t c) {
                uint32_t keep = 0xFFFFu;
                if (c == c0) keep &= 0xFFFFu << (r0 & 15);
                if (c == c1) keep &= 0xFFFFu >> (15 - ((lim - 1) & 15));
                return m & keep;
            };
            for (uint64_t t = W.te_any & span; t; t &= t - 1) {
                const uint32_t c = (uint32_t)__builtin_ctzll(t);
                if (in_range(rl(W.te, c), c)) return 0;  // transfer-encoding: the classifier frames the body
            }
            for (uint64_t t = W.cl_any & span; t;) {
                const uint32_t c = 63 - (uint32_t)__builtin_clzll(t);
                const uint32_t m = in_range(rl(W.cl, c), c);
                if (m) {
                    last_cl = W.wa + 16ull * c + (31 - __builtin_clz(m)) - (uint64_t)W.A;
                    break;
                }
                t &= ~(1ull << c);
            }
        }
        if (found) {
            e = W.wa + re - (uint64_t)W.A;
            break;
        }
        if (W.wa + kWinBytes >= (uint64_t)W.A + W.n) return 0;  // no "\r\n\r\n": incomplete
        x = s_end - (uint64_t)W.A;
        twin_load(W, W.wa + kNextWin);  // (s_end - 16: the scan goes on at its byte 16)
    }
    uint64_t cl = 0;
    if (last_cl != ~0ull) {  // strtoull: leading spaces, optional sign, digits
        uint64_t i = last_cl + 15;
        while (i < W.n) {
            const uint32_t c = tbyte(W, i);
            if (!(c == ' ' || (c >= 0x09 && c <= 0x0D))) break;
            i++;
        }
        bool neg = false;
        if (i < W.n) {
            const uint32_t c = tbyte(W, i);
            if (c == '+' || c == '-') { neg = c == '-'; i++; }
        }
        uint64_t v = 0;
        bool over = false;
        for (; i < W.n; i++) {
            const uint32_t d = tbyte(W, i) - '0';
            if (d > 9) break;
            if (v > (~0ull - d) / 10) over = true;
            v = over ? ~0ull : v * 10 + d;
        }
        cl = neg ? 0 - v : v;
    }
    const uint64_t head_end = e + 4;
    if (cl > W.n - head_end) return 0;
    return head_end + cl;
}

// NextMcText on the window (next_mc_text's semantics): the tokens of the line
// from the separator masks when the line lies in one window, else byte by byte
__device__ __forceinline__ uint64_t tnext_mc_text(TWin &W, uint64_t p) {
    const uint64_t lf = tfind_crlf(W, p);
    if (lf >= W.n) return 0;
    uint64_t t0 = 0, t0e = 0, t4 = 0, t4e = 0;
    uint32_t nt = 0;
    bool in = false;
    twin_at(W, p);
    if ((uint64_t)W.A + lf <= W.wa + kWinBytes - 1 && (uint64_t)W.A + p >= W.wa) {
        const uint32_t x0 = (uint32_t)((uint64_t)W.A + p - W.wa), x1 = (uint32_t)((uint64_t)W.A + lf - W.wa);
        for (uint32_t c = x0 >> 4; c <= ((x1 - 1) >> 4) && x1 > x0 && nt <= 4; c++) {
            const uint32_t lo = c == (x0 >> 4) ? (x0 & 15) : 0u, hi = c == (x1 >> 4) ? (x1 & 15) : 16u;
            const uint32_t range = (0xFFFFu << lo) & (0xFFFFu >> (16 - hi));
            const uint32_t tok = ~rl(W.sp, c) & range;
            const uint32_t inb = in ? 1u : 0u;
            uint32_t starts = tok & ~((tok << 1) | (lo == 0 ? inb : 0u)) & range;
            uint32_t stops = ~tok & ((tok << 1) | (lo == 0 ? inb : 0u)) & range;
            while ((starts | stops) && nt <= 4) {
                const uint32_t k = __builtin_ctz(starts | stops);
                const uint64_t pos = W.wa + 16ull * c + k - (uint64_t)W.A;
                if ((starts >> k) & 1) {
                    if (nt == 0) t0 = pos;
                    if (nt == 4) t4 = pos;
                    in = true;
                    starts &= starts - 1;
                } else {
                    if (nt == 0) t0e = pos;
                    if (nt == 4) t4e = pos;
                    nt++;
                    in = false;
                    stops &= stops - 1;
                }
            }
        }
    } else {
        // a line over a window: bytes.Fields byte by byte (shim.cc SpaceLen)
        for (uint64_t i = p; i < lf;) {
            const uint32_t c = tbyte(W, i);
            uint32_t sp = 0;
            if (c == ' ' || (c >= 0x09 && c <= 0x0D)) sp = 1;
            else if (c >= 0xC2 && c <= 0xE3 && i + 1 < lf) {
                const uint32_t c1 = tbyte(W, i + 1);
                if (c == 0xC2) sp = (c1 == 0x85 || c1 == 0xA0) ? 2 : 0;
                else if (i + 2 < lf) {
                    const uint32_t c2 = tbyte(W, i + 2);
                    if (c == 0xE1) sp = (c1 == 0x9A && c2 == 0x80) ? 3 : 0;
                    else if (c == 0xE2 && c1 == 0x80) sp = ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF) ? 3 : 0;
                    else if (c == 0xE2 && c1 == 0x81) sp = c2 == 0x9F ? 3 : 0;
                    else if (c == 0xE3) sp = (c1 == 0x80 && c2 == 0x80) ? 3 : 0;
                }
            }
            if (sp) {
                if (in) {
                    if (nt == 0) t0e = i;
                    if (nt == 4) t4e = i;
                    nt++;
                }
                in = false;
                i += sp;
            } else {
                if (!in) {
                    if (nt == 0) t0 = i;
                    if (nt == 4) t4 = i;
                    in = true;
                }
                i++;
            }
            if (nt > 4) break;
        }
    }
    if (in && nt <= 4) {
        if (nt == 0) t0e = lf;
        if (nt == 4) t4e = lf;
        nt++;
    }
    uint64_t next = lf + 2;
    bool storage = false;
    if (nt >= 1) {
        const uint64_t k = t0e - t0;
        if (k == 3 || k == 6 || k == 7) {
            const uint32_t a = tword(W, t0), b = k > 4 ? tword(W, t0 + 4) : 0u;
            const uint32_t a3 = a & 0xFFFFFFu;
            storage = (k == 3 && (a3 == 0x746573u || a3 == 0x646461u || a3 == 0x736163u)) ||      // set add cas
                      (k == 6 && a == 0x65707061u && (b & 0xFFFFu) == 0x646eu) ||                // append
                      (k == 7 && ((a == 0x6c706572u && (b & 0xFFFFFFu) == 0x656361u) ||           // replace
                                  (a == 0x70657270u && (b & 0xFFFFFFu) == 0x646e65u)));          // prepend
        }
    }
    if (storage) {
        if (nt < 5) return 0;
        uint64_t i = t4;
        bool neg = false;
        if (i < t4e) {
            const uint32_t c = tbyte(W, i);
            if (c == '+' || c == '-') { neg = c == '-'; i++; }
        }
        if (i >= t4e) return 0;
        uint64_t v = 0;
        for (; i < t4e; i++) {
            const uint32_t d = tbyte(W, i) - '0';
            if (d > 9) return 0;
            v = v * 10 + d;
            if (v > (1ull << 40)) return 0;
        }
        if (neg && v) return 0;
        next += v + 2;
    }
    return next <= W.n ? next : 0;
}

__device__ __forceinline__ bool text_stream(const DevConn &c, uint32_t first) {
    if (c.proto == PROTO_HTTP || c.proto == PROTO_R2D2) return true;
    if (c.proto != PROTO_MEMCACHE) return false;
    const uint32_t mode = c.flags & 3;
    return mode == 1 || (mode == 0 && first < 0x80);
}

}  // namespace

// 4 waves per SIMD (<= 128 VGPRs; left to itself the compiler takes 130 and
// 3 waves: 1M HTTP requests in 16k streams 6.24 -> 6.28 ms, memcached text
// 9.05 -> 8.59 ms).  One lane per stream.  Slots [s * max_frames, (s + 1) * max_frames) of the
// outputs belong to stream s: frame k starts at frame_off (an arena offset)
// and is handed frame_len bytes (to the stream's end); conn_out = the
// stream's connection; slots past nframes[s] get length 0 and connection
// ~0 (answered UNSUPPORTED by the classifiers, which may run over every slot).
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(4))) void frame_streams_kernel(const uint8_t *__restrict__ arena, uint64_t arena_len,
                                                               const uint64_t *__restrict__ s_off,
                                                               const uint32_t *__restrict__ s_len,
                                                               const uint32_t *__restrict__ s_conn, uint32_t n,
                                                               const DevConn *__restrict__ conns, uint32_t nconns,
                                                               uint32_t max_frames, uint64_t *__restrict__ frame_off,
                                                               uint32_t *__restrict__ frame_len,
                                                               uint32_t *__restrict__ conn_out,
                                                               uint32_t *__restrict__ nframes, uint32_t text_waves) {
    for (uint32_t s = blockIdx.x * kBlock + threadIdx.x; s < n; s += gridDim.x * kBlock) {
        const uint64_t so = s_off[s];
        const uint32_t sl = s_len[s];
        const uint32_t ci = s_conn[s];
        const size_t slot0 = (size_t)s * max_frames;
        uint32_t k = 0;
        if (l7_in_arena(so, sl, arena_len) && sl > 0 && ci < nconns) {
            const DevConn c = conns[ci];
            Stream S{arena + so, sl, ~0ull, make_uint4(0, 0, 0, 0)};
            uint32_t mode = c.flags & 3;  // memcached: the connection's parser, else the first byte's
            if (c.proto == PROTO_MEMCACHE && mode == 0) mode = sbyte(S, 0) >= 0x80 ? 2 : 1;
            if (text_waves && text_stream(c, sbyte(S, 0))) continue;  // frame_text_kernel walks it
            for (uint64_t p = 0; p < S.n && k < max_frames;) {
                frame_off[slot0 + k] = so + p;
                frame_len[slot0 + k] = (uint32_t)(S.n - p);
                conn_out[slot0 + k] = ci;
                k++;
                uint64_t q = 0;
                switch (c.proto) {
                case PROTO_KAFKA: q = next_kafka(S, p); break;
                case PROTO_HTTP: q = next_http(S, p); break;
                case PROTO_R2D2: q = next_line(S, p); break;
                case PROTO_CASSANDRA: q = next_cassandra(S, p); break;
                case PROTO_MEMCACHE: q = mode == 2 ? next_mc_binary(S, p) : next_mc_text(S, p); break;
                default: break;
                }
                if (q <= p) break;
                p = q;
            }
        } else if (sl > 0 || ci >= nconns) {  // out of contract / unknown connection: one slot, answered as is
            frame_off[slot0] = so;
            frame_len[slot0] = sl;
            conn_out[slot0] = ci;
            k = max_frames ? 1 : 0;
        }
        nframes[s] = k;
        for (uint32_t j = k; j < max_frames; j++) {
            frame_off[slot0 + j] = 0;
            frame_len[slot0 + j] = 0;
            conn_out[slot0 + j] = ~0u;
        }
    }
}


// The text streams (HTTP, memcached text, r2d2), a wave per stream: the same
// frames as frame_streams_kernel's one-lane walk, whose other streams it skips.
constexpr int kTBlock = 256;
__global__ __launch_bounds__(kTBlock) void frame_text_kernel(const uint8_t *__restrict__ arena, uint64_t arena_len,
                                                             const uint64_t *__restrict__ s_off,
                                                             const uint32_t *__restrict__ s_len,
                                                             const uint32_t *__restrict__ s_conn, uint32_t n,
                                                             const DevConn *__restrict__ conns, uint32_t nconns,
                                                             uint32_t max_frames, uint64_t *__restrict__ frame_off,
                                                             uint32_t *__restrict__ frame_len,
                                                             uint32_t *__restrict__ conn_out,
                                                             uint32_t *__restrict__ nframes) {
    const uint32_t lane = threadIdx.x & 63;
    const uint32_t waves = gridDim.x * (kTBlock / 64);
    const uint32_t wave0 = (uint32_t)__builtin_amdgcn_readfirstlane((int)(blockIdx.x * (kTBlock / 64) + (threadIdx.x >> 6)));
    for (uint32_t s = wave0; s < n; s += waves) {
        // the stream's metadata as wave-uniform values (SGPRs): the walk below
        // is scalar code, its branches scalar branches
        const uint64_t so0 = s_off[s];
        const uint64_t so = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)so0) |
                            (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(so0 >> 32)) << 32;
        const uint32_t sl = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_len[s]);
        const uint32_t ci = (uint32_t)__builtin_amdgcn_readfirstlane((int)s_conn[s]);
        if (!(l7_in_arena(so, sl, arena_len) && sl > 0 && ci < nconns)) continue;  // (the lane kernel's)
        const DevConn c0 = conns[ci];
        DevConn c;
        c.ruleset = __builtin_amdgcn_readfirstlane(c0.ruleset);
        const uint32_t pf = (uint32_t)__builtin_amdgcn_readfirstlane((int)((uint32_t)c0.proto | (uint32_t)c0.flags << 8));
        c.proto = (uint8_t)pf;
        c.flags = (uint8_t)(pf >> 8);
        c.skey = 0;
        if (!text_stream(c, (uint32_t)__builtin_amdgcn_readfirstlane((int)arena[so]))) continue;
        TWin W;
        W.A = arena + so;
        W.n = sl;
        W.wa = ~0ull;
        W.want_sp = c.proto == PROTO_MEMCACHE;
        W.want_http = c.proto == PROTO_HTTP;
        W.nwa = ~0ull;
        FPH(W.ph_load = 0; W.ph_n = 0; const uint64_t ts_ = __builtin_amdgcn_s_memtime();)
        const size_t slot0 = (size_t)s * max_frames;
        uint32_t k = 0;
        for (uint64_t p = 0; p < W.n && k < max_frames;) {
            if (lane == 0) {
                frame_off[slot0 + k] = so + p;
                frame_len[slot0 + k] = (uint32_t)(W.n - p);
                conn_out[slot0 + k] = ci;
            }
            k++;
            const uint64_t q = c.proto == PROTO_HTTP ? tnext_http(W, p)
                             : c.proto == PROTO_R2D2 ? ((void)0, [&] { const uint64_t lf = tfind_crlf(W, p); return lf >= W.n ? 0ull : lf + 2; }())
                             : tnext_mc_text(W, p);
            if (q <= p) break;
            p = q;
        }
        if (lane == 0) nframes[s] = k;
        FPH(if (lane == 0) {
            atomicAdd(&g_fphase[0], (unsigned long long)W.ph_load);
            atomicAdd(&g_fphase[1], (unsigned long long)(__builtin_amdgcn_s_memtime() - ts_));
            atomicAdd(&g_fphase[2], (unsigned long long)W.ph_n);
            atomicAdd(&g_fphase[3], (unsigned long long)k);
            atomicAdd(&g_fphase[4], 1ull);
        })
        for (uint32_t j = k + lane; j < max_frames; j += 64) {
            frame_off[slot0 + j] = 0;
            frame_len[slot0 + j] = 0;
            conn_out[slot0 + j] = ~0u;
        }
    }
}

hipError_t FramePhaseTimes(uint64_t *out, bool reset) {
#ifdef L7G_FRAME_PHASES
    hipError_t rc = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_fphase), sizeof(uint64_t) * 8);
    if (rc == hipSuccess && reset) {
        const uint64_t z[8] = {};
        rc = hipMemcpyToSymbol(HIP_SYMBOL(g_fphase), z, sizeof z);
    }
    return rc;
#else
    (void)out;
    (void)reset;
    return hipErrorNotSupported;
#endif
}

hipError_t LaunchFrameStreams(const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off, const uint32_t *s_len,
                              const uint32_t *s_conn, uint32_t n, const DevConn *conns, uint32_t nconns,
                              uint32_t max_frames, uint64_t *frame_off, uint32_t *frame_len, uint32_t *conn_out,
                              uint32_t *nframes, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = min((n + kBlock - 1) / kBlock, 65536u);
    hipLaunchKernelGGL(frame_streams_kernel, dim3(blocks), dim3(kBlock), 0, stream, arena, arena_len, s_off, s_len,
                       s_conn, n, conns, nconns, max_frames, frame_off, frame_len, conn_out, nframes, 1u);
    const uint32_t tblocks = min((n + kTBlock / 64 - 1) / (kTBlock / 64), 65536u);
    hipLaunchKernelGGL(frame_text_kernel, dim3(tblocks), dim3(kTBlock), 0, stream, arena, arena_len, s_off, s_len,
                       s_conn, n, conns, nconns, max_frames, frame_off, frame_len, conn_out, nframes);
    return hipGetLastError();
}

}  // namespace l7
