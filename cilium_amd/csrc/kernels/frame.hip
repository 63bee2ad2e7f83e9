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
                                                               uint32_t *__restrict__ nframes) {
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

hipError_t LaunchFrameStreams(const uint8_t *arena, uint64_t arena_len, const uint64_t *s_off, const uint32_t *s_len,
                              const uint32_t *s_conn, uint32_t n, const DevConn *conns, uint32_t nconns,
                              uint32_t max_frames, uint64_t *frame_off, uint32_t *frame_len, uint32_t *conn_out,
                              uint32_t *nframes, hipStream_t stream) {
    if (n == 0) return hipSuccess;
    const uint32_t blocks = min((n + kBlock - 1) / kBlock, 65536u);
    hipLaunchKernelGGL(frame_streams_kernel, dim3(blocks), dim3(kBlock), 0, stream, arena, arena_len, s_off, s_len,
                       s_conn, n, conns, nconns, max_frames, frame_off, frame_len, conn_out, nframes);
    return hipGetLastError();
}

}  // namespace l7
