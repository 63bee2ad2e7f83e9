// Lane-serial Kafka wire decoding helpers shared by the classification kernel
// (kafka_classify.hip) and the compressed-set kernel (kafka_inflate.hip):
// the per-lane 16-byte chunk cursor, io.ReadFull / LimitReader reads
// (vendor/github.com/optiopay/kafka/proto/serialization.go:19-203), big-endian
// fields and CRC32-IEEE (hash/crc32.ChecksumIEEE, slicing-by-8 LDS tables).
// Product code.
#pragma once
#include <hip/hip_runtime.h>

#include <stdint.h>

#include "gmem.h"

namespace l7 {
namespace {

constexpr uint32_t kMaxParseBuf = 6553500;
constexpr int kCrcSlices = 8;
#define L7G_KAFKA_CRCSTREAMS 1  // independent CRC chains per 64-byte batch (2 and 4 measured slower, round 3)
// Shift tables after the 8 slicing tables: Zn[j][b] = T_{n-1-j}[b], so that
// crc(v, n zero bytes) = Zn[0][v & 0xFF] ^ ... ^ Zn[3][v >> 24] (the register
// state is linear: crc(c, A || B) = crc(crc(c, A), 0^|B|) ^ crc(0, B)).
constexpr int kCrcZ32 = 8 * 256, kCrcZ48 = 12 * 256, kCrcZ16 = 16 * 256;
constexpr int kCrcTables = L7G_KAFKA_CRCSTREAMS == 1 ? 8 : L7G_KAFKA_CRCSTREAMS == 2 ? 12 : 20;
// The tables of one workgroup: thread t < 256 fills entry t of each.
__device__ __forceinline__ void crc_tables_init(uint32_t *tab, uint32_t t) {
    if (t < 256) {
        uint32_t c = t;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        tab[t] = c;
    }
    __syncthreads();
    if (t < 256) {
        uint32_t v = tab[t];
        for (int k = 1; k < (kCrcTables == 8 ? 8 : kCrcTables == 12 ? 32 : 48); k++) {
            v = (v >> 8) ^ tab[v & 0xFF];  // T_k[t]
            if (k < 8) tab[k * 256 + t] = v;
            if (kCrcTables >= 12 && k >= 28 && k < 32) tab[kCrcZ32 + (31 - k) * 256 + t] = v;
            if (kCrcTables >= 20 && k >= 44) tab[kCrcZ48 + (47 - k) * 256 + t] = v;
            if (kCrcTables >= 20 && k >= 12 && k < 16) tab[kCrcZ16 + (15 - k) * 256 + t] = v;
        }
    }
    __syncthreads();
}
__device__ __forceinline__ uint32_t crc_slice8(const uint32_t *tab, uint32_t lo, uint32_t hi) {
    return tab[7 * 256 + (lo & 0xFF)] ^ tab[6 * 256 + ((lo >> 8) & 0xFF)] ^ tab[5 * 256 + ((lo >> 16) & 0xFF)] ^
           tab[4 * 256 + (lo >> 24)] ^ tab[3 * 256 + (hi & 0xFF)] ^ tab[2 * 256 + ((hi >> 8) & 0xFF)] ^
           tab[1 * 256 + ((hi >> 16) & 0xFF)] ^ tab[hi >> 24];
}
__device__ __forceinline__ uint32_t crc_shift(const uint32_t *z, uint32_t v) {
    return z[v & 0xFF] ^ z[256 + ((v >> 8) & 0xFF)] ^ z[512 + ((v >> 16) & 0xFF)] ^ z[768 + (v >> 24)];
}
constexpr uint32_t kInf = 0xFFFFFFFFu;

// Per-lane byte cursor: the decoders walk their request forward, so each lane
// keeps the aligned block it last touched in registers and serves field bytes
// from it.  CurT<4>: one 16-byte chunk (one dwordx4 load replaces up to 16 byte
// loads); CurT<16>: a 64-byte block (four dwordx4 loads issued together, so a
// message header, a topic entry or a request header is one memory latency, not
// two or three).  A block that holds a request byte never leaves that byte's
// page, so the aligned over-read is safe for any arena alignment.
template <int NW>
struct CurT;
template <>
struct CurT<4> {
    uintptr_t line;  // address of the cached block (~0 = none)
    uint32_t w0, w1, w2, w3;  // scalars, not an array: a selected array element would put Cur in scratch
};
template <>
struct CurT<8> {
    uintptr_t line;
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7;
};
template <>
struct CurT<16> {
    uintptr_t line;
    uint32_t w0, w1, w2, w3, w4, w5, w6, w7, w8, w9, w10, w11, w12, w13, w14, w15;
};
using Cur = CurT<4>;
template <int NW>
__device__ __forceinline__ void cur_fill(CurT<NW> &c, uintptr_t a) {
    const uintptr_t ln = a & ~(uintptr_t)(NW * 4 - 1);
    if (ln != c.line) {
        if constexpr (NW == 4) {
            const uint4 v = gload16(ln);
            c.w0 = v.x; c.w1 = v.y; c.w2 = v.z; c.w3 = v.w;
        } else if constexpr (NW == 8) {
            const uint4 v0 = gload16(ln), v1 = gload16(ln + 16);
            c.w0 = v0.x; c.w1 = v0.y; c.w2 = v0.z; c.w3 = v0.w;
            c.w4 = v1.x; c.w5 = v1.y; c.w6 = v1.z; c.w7 = v1.w;
        } else {
            const uint4 v0 = gload16(ln), v1 = gload16(ln + 16), v2 = gload16(ln + 32), v3 = gload16(ln + 48);
            c.w0 = v0.x; c.w1 = v0.y; c.w2 = v0.z; c.w3 = v0.w;
            c.w4 = v1.x; c.w5 = v1.y; c.w6 = v1.z; c.w7 = v1.w;
            c.w8 = v2.x; c.w9 = v2.y; c.w10 = v2.z; c.w11 = v2.w;
            c.w12 = v3.x; c.w13 = v3.y; c.w14 = v3.z; c.w15 = v3.w;
        }
        c.line = ln;
    }
}
// word i of the block, 0 past its end (values are copied out before they are
// selected: a select between struct members becomes a select between their
// addresses, i.e. a scratch array)
template <int NW>
__device__ __forceinline__ uint32_t cur_wordi(const CurT<NW> &c, uint32_t i) {
    if constexpr (NW == 4) {
        const uint32_t a = c.w0, b = c.w1, d = c.w2, e = c.w3;
        return i < 2 ? (i == 0 ? a : b) : i == 2 ? d : i == 3 ? e : 0u;
    } else if constexpr (NW == 8) {
        const uint32_t x0 = c.w0, x1 = c.w1, x2 = c.w2, x3 = c.w3, x4 = c.w4, x5 = c.w5, x6 = c.w6, x7 = c.w7;
        const uint32_t lo4 = (i & 2) ? ((i & 1) ? x3 : x2) : ((i & 1) ? x1 : x0);
        const uint32_t hi4 = (i & 2) ? ((i & 1) ? x7 : x6) : ((i & 1) ? x5 : x4);
        return i < 8 ? ((i & 4) ? hi4 : lo4) : 0u;
    } else {
        const uint32_t x0 = c.w0, x1 = c.w1, x2 = c.w2, x3 = c.w3, x4 = c.w4, x5 = c.w5, x6 = c.w6, x7 = c.w7;
        const uint32_t x8 = c.w8, x9 = c.w9, x10 = c.w10, x11 = c.w11, x12 = c.w12, x13 = c.w13, x14 = c.w14,
                       x15 = c.w15;
        const uint32_t lo4 = (i & 2) ? ((i & 1) ? x3 : x2) : ((i & 1) ? x1 : x0);
        const uint32_t hi4 = (i & 2) ? ((i & 1) ? x7 : x6) : ((i & 1) ? x5 : x4);
        const uint32_t lo8 = (i & 2) ? ((i & 1) ? x11 : x10) : ((i & 1) ? x9 : x8);
        const uint32_t hi8 = (i & 2) ? ((i & 1) ? x15 : x14) : ((i & 1) ? x13 : x12);
        const uint32_t v = (i & 8) ? ((i & 4) ? hi8 : lo8) : ((i & 4) ? hi4 : lo4);
        return i < 16 ? v : 0u;
    }
}
template <int NW>
__device__ __forceinline__ uint32_t cur_word(const CurT<NW> &c, uint32_t k) {
    return cur_wordi(c, k >> 2);
}
template <int NW>
__device__ __forceinline__ uint32_t cur_byte(CurT<NW> &c, const uint8_t *p) {
    const uintptr_t a = (uintptr_t)p;
    cur_fill(c, a);
    const uint32_t k = (uint32_t)(a & (NW * 4 - 1));
    return (cur_word(c, k) >> ((k & 3) * 8)) & 0xFFu;
}

template <class C>
struct KDecT {
    const uint8_t *b;
    uint32_t pos, end;
    int32_t limit;  // LimitReader remaining, -1 = none (a set is at most kMaxParseBuf)
    int err;        // 0 ok, 1 EOF, 2 ErrUnexpectedEOF, 3 other
    C *c;
};
using KDec = KDecT<Cur>;

template <class D>
__device__ __forceinline__ uint32_t kavail(const D &d) {
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint32_t)d.limit < a) a = (uint32_t)d.limit;
    return a;
}
// io.ReadFull(r, buf[:n]); returns start offset, sets d.err on a short read
template <class D>
__device__ __forceinline__ uint32_t kread(D &d, uint32_t n) {
    uint32_t at = d.pos;
    if (n == 0) return at;
    uint32_t a = kavail(d);
    if (a == 0) { d.err = 1; return at; }
    uint32_t take = a < n ? a : n;
    d.pos += take;
    if (d.limit >= 0) d.limit -= (int32_t)take;
    if (take < n) d.err = 2;
    return at;
}
// Big-endian n-byte field (n = 1, 2, 4 or 8).  A field inside the cached
// block is cut out of two adjacent words (v_alignbyte) and byte-swapped
// (v_perm); one straddling two blocks is read byte by byte.
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0, x, 0x00010203u); }
template <int NW>
__device__ __forceinline__ uint64_t be_load(CurT<NW> &c, const uint8_t *p, int n) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t k = (uint32_t)(a & (NW * 4 - 1));
    if (n <= 4 && k + (uint32_t)n <= NW * 4) {
        cur_fill(c, a);
        const uint32_t i = k >> 2;
        const uint32_t lo = cur_wordi(c, i), hi = cur_wordi(c, i + 1);
        const uint32_t v = bswap32(__builtin_amdgcn_alignbyte(hi, lo, k & 3));  // bytes k..k+3, big-endian
        return n == 4 ? v : v >> (32 - 8 * n);
    }
    if (n == 8) return (be_load(c, p, 4) << 32) | be_load(c, p + 4, 4);
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | cur_byte(c, p + i);
    return v;
}
template <class D>
__device__ __forceinline__ int64_t dec_int(D &d, int n) {
    if (d.err) return 0;
    uint32_t at = kread(d, (uint32_t)n);
    if (d.err) return 0;
    uint64_t v = be_load(*d.c, d.b + at, n);
    return n == 1 ? (int64_t)(int8_t)v : n == 2 ? (int64_t)(int16_t)v : n == 4 ? (int64_t)(int32_t)v : (int64_t)v;
}
// A field whose value is not needed: only the read (and its errors) matter.
template <class D>
__device__ __forceinline__ void dec_skip(D &d, int n) {
    if (d.err) return;
    kread(d, (uint32_t)n);
}
// DecodeString -> (off, len); len < 1 => ""
template <class D>
__device__ __forceinline__ void dec_string(D &d, uint32_t &off, uint32_t &len) {
    off = 0; len = 0;
    if (d.err) return;
    int16_t sl = (int16_t)dec_int(d, 2);
    if (d.err || sl < 1) return;
    uint32_t at = kread(d, (uint32_t)sl);
    if (d.err) return;
    off = at; len = (uint32_t)sl;
}
// DecodeArrayLen(nullable): -1 null; sets bad on ErrInvalidArrayLen
template <class D>
__device__ __forceinline__ int32_t dec_arraylen(D &d, bool nullable, bool &bad) {
    int32_t l = (int32_t)dec_int(d, 4);
    bad = false;
    if (l < 0) { if (nullable) return -1; bad = true; return 0; }
    if ((uint32_t)l > kMaxParseBuf) { bad = true; return 0; }
    return l;
}
template <class D>
__device__ __forceinline__ void dec_bytes(D &d) {
    if (d.err) return;
    int32_t sl = (int32_t)dec_int(d, 4);
    if (d.err || sl < 1) return;
    if ((uint32_t)sl > kMaxParseBuf) { d.err = 3; return; }
    kread(d, (uint32_t)sl);
}

// CRC32-IEEE (hash/crc32.ChecksumIEEE), slicing-by-8: tab holds 8 LDS tables
// of 256 entries; the body advances 8 aligned bytes per step with eight
// independent table reads, so the serial chain is one step per 8 bytes.
__device__ __forceinline__ uint32_t crc32_ieee(const uint32_t *tab, Cur &cur, const uint8_t *p, uint32_t n) {
    uint32_t c = 0xFFFFFFFFu;
    uint32_t i = 0;
    for (; i < n && (((uintptr_t)(p + i)) & 15); i++) c = tab[(c ^ cur_byte(cur, p + i)) & 0xFF] ^ (c >> 8);
    // Bulk: 64 aligned bytes per batch, four dwordx4 loads issued together so
    // one memory latency covers 8 slicing steps (a lane walks its message
    // alone; back-to-back dependent loads were the kernel's critical path).
    for (; i + 64 <= n; i += 64) {
        const uint4 *q = reinterpret_cast<const uint4 *>(p + i);
        uint4 v[4];
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = q[j];
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const uint4 &x = v[j >> 1];
            const uint32_t lo = ((j & 1) ? x.z : x.x) ^ c, hi = (j & 1) ? x.w : x.y;
            c = tab[7 * 256 + (lo & 0xFF)] ^ tab[6 * 256 + ((lo >> 8) & 0xFF)] ^ tab[5 * 256 + ((lo >> 16) & 0xFF)] ^
                tab[4 * 256 + (lo >> 24)] ^ tab[3 * 256 + (hi & 0xFF)] ^ tab[2 * 256 + ((hi >> 8) & 0xFF)] ^
                tab[1 * 256 + ((hi >> 16) & 0xFF)] ^ tab[hi >> 24];
        }
    }
    for (; i + 8 <= n; i += 8) {
        const uintptr_t a = (uintptr_t)(p + i);
        cur_fill(cur, a);
        const uint32_t k = (uint32_t)(a & 15);
        const uint32_t w0 = cur.w0, w1 = cur.w1, w2 = cur.w2, w3 = cur.w3;
        const uint32_t lo = (k ? w2 : w0) ^ c, hi = k ? w3 : w1;
        c = tab[7 * 256 + (lo & 0xFF)] ^ tab[6 * 256 + ((lo >> 8) & 0xFF)] ^ tab[5 * 256 + ((lo >> 16) & 0xFF)] ^
            tab[4 * 256 + (lo >> 24)] ^ tab[3 * 256 + (hi & 0xFF)] ^ tab[2 * 256 + ((hi >> 8) & 0xFF)] ^
            tab[1 * 256 + ((hi >> 16) & 0xFF)] ^ tab[hi >> 24];
    }
    for (; i < n; i++) c = tab[(c ^ cur_byte(cur, p + i)) & 0xFF] ^ (c >> 8);
    return ~c;
}


// One slicing-by-8 step over (lo ^ c, hi), and one slicing-by-4 step over a
// word x = w ^ c, with every table lookup in flight before the single wait.
// (Written out because the compiler, short of registers at 6 waves per SIMD,
// issued the tail loop's eight lookups one or two at a time, each behind its
// own LDS wait.)  tabaddr: the LDS address of table 0; table k is k KiB on.
__device__ __forceinline__ uint32_t crc_step8(uint32_t tabaddr, uint32_t lo, uint32_t hi) {
    const uint32_t a0 = tabaddr + ((lo & 0xFF) << 2), a1 = tabaddr + (((lo >> 8) & 0xFF) << 2),
                   a2 = tabaddr + (((lo >> 16) & 0xFF) << 2), a3 = tabaddr + ((lo >> 24) << 2),
                   a4 = tabaddr + ((hi & 0xFF) << 2), a5 = tabaddr + (((hi >> 8) & 0xFF) << 2),
                   a6 = tabaddr + (((hi >> 16) & 0xFF) << 2), a7 = tabaddr + ((hi >> 24) << 2);
    uint32_t r0, r1, r2, r3, r4, r5, r6, r7;
    asm volatile(
        "ds_read_b32 %0, %8 offset:7168\n\tds_read_b32 %1, %9 offset:6144\n\t"
        "ds_read_b32 %2, %10 offset:5120\n\tds_read_b32 %3, %11 offset:4096\n\t"
        "ds_read_b32 %4, %12 offset:3072\n\tds_read_b32 %5, %13 offset:2048\n\t"
        "ds_read_b32 %6, %14 offset:1024\n\tds_read_b32 %7, %15\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3), "=&v"(r4), "=&v"(r5), "=&v"(r6), "=&v"(r7)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3), "v"(a4), "v"(a5), "v"(a6), "v"(a7)
        : "memory");
    return (r0 ^ r1) ^ (r2 ^ r3) ^ (r4 ^ r5) ^ (r6 ^ r7);
}
__device__ __forceinline__ uint32_t crc_step4(uint32_t tabaddr, uint32_t x) {
    const uint32_t a0 = tabaddr + ((x & 0xFF) << 2), a1 = tabaddr + (((x >> 8) & 0xFF) << 2),
                   a2 = tabaddr + (((x >> 16) & 0xFF) << 2), a3 = tabaddr + ((x >> 24) << 2);
    uint32_t r0, r1, r2, r3;
    asm volatile(
        "ds_read_b32 %0, %4 offset:3072\n\tds_read_b32 %1, %5 offset:2048\n\t"
        "ds_read_b32 %2, %6 offset:1024\n\tds_read_b32 %3, %7\n\t"
        "s_waitcnt lgkmcnt(0)"
        : "=&v"(r0), "=&v"(r1), "=&v"(r2), "=&v"(r3)
        : "v"(a0), "v"(a1), "v"(a2), "v"(a3)
        : "memory");
    return (r0 ^ r1) ^ (r2 ^ r3);
}
// The CRC over r <= 3 bytes (x: those bytes little-endian, upper bytes ignored):
// c' = (c >> 8r) ^ sum_j T[r-1-j][(c >> 8j ^ b_j) & 0xFF], the lookups in flight
// together (1 <= r <= 3).
__device__ __forceinline__ uint32_t crc_bytes3(uint32_t tabaddr, uint32_t c, uint32_t x, uint32_t r) {
    const uint32_t y = c ^ x;
    const uint32_t a0 = tabaddr + ((r - 1) << 10) + ((y & 0xFF) << 2);
    const uint32_t a1 = tabaddr + ((r - 2) << 10) + (((y >> 8) & 0xFF) << 2);
    const uint32_t a2 = tabaddr + (((y >> 16) & 0xFF) << 2);
    const uint32_t b0 = r >= 1 ? a0 : tabaddr, b1 = r >= 2 ? a1 : tabaddr, b2 = r >= 3 ? a2 : tabaddr;
    uint32_t r0, r1, r2;
    asm volatile("ds_read_b32 %0, %3\n\tds_read_b32 %1, %4\n\tds_read_b32 %2, %5\n\ts_waitcnt lgkmcnt(0)"
                 : "=&v"(r0), "=&v"(r1), "=&v"(r2)
                 : "v"(b0), "v"(b1), "v"(b2)
                 : "memory");
    return (c >> (8 * r)) ^ r0 ^ (r >= 2 ? r1 : 0u) ^ (r >= 3 ? r2 : 0u);
}
// little-endian bytes k .. k+3 of the cursor's chunk (k <= 12)
__device__ __forceinline__ uint32_t cur_word_at(const Cur &c, uint32_t k) {
    const uint32_t w0 = c.w0, w1 = c.w1, w2 = c.w2, w3 = c.w3;
    const uint32_t i = k >> 2;
    const uint32_t lo = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
    const uint32_t hi = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
    return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
}

// CRC32-IEEE of r bytes at byte j of the 16-byte chunk v (j + r <= 16): 8-,
// 4- and <= 3-byte slicing steps, each step's lookups in flight together.
__device__ __forceinline__ uint32_t crc_chunk_span(uint32_t tabaddr, uint32_t c, const uint4 &v, uint32_t j, uint32_t r) {
    auto word_at = [&](uint32_t k) -> uint32_t {  // little-endian bytes k .. k+3 (k <= 12)
        const uint32_t i = k >> 2;
        const uint32_t lo = i == 0 ? v.x : i == 1 ? v.y : i == 2 ? v.z : v.w;
        const uint32_t hi = i == 0 ? v.y : i == 1 ? v.z : i == 2 ? v.w : 0u;
        return __builtin_amdgcn_alignbyte(hi, lo, k & 3);
    };
    if (j == 0 && r == 16) {
        c = crc_step8(tabaddr, v.x ^ c, v.y);
        return crc_step8(tabaddr, v.z ^ c, v.w);
    }
    uint32_t i = 0;
    if (r >= 8) {
        c = crc_step8(tabaddr, word_at(j) ^ c, word_at(j + 4));
        i = 8;
    }
    if (r - i >= 4) {
        c = crc_step4(tabaddr, word_at(j + i) ^ c);
        i += 4;
    }
    if (i < r) c = crc_bytes3(tabaddr, c, word_at(j + i), r - i);
    return c;
}
// CRC32-IEEE of [p, p + n) in global memory: the aligned 16-byte chunks that
// hold it, 64 bytes per group, the next group's loads issued before the
// current one is hashed (two groups in flight per lane, so a lane walking a
// message waits about one memory latency per 64 bytes less).
__device__ __forceinline__ uint32_t crc32_ieee_global(uint32_t tabaddr, const uint8_t *p, uint32_t n) {
    uint32_t c = 0xFFFFFFFFu;
    if (n == 0) return ~c;
    const uint64_t a = (uint64_t)(uintptr_t)p, ab = a & ~15ull;
    const uint32_t j0 = (uint32_t)(a & 15);
    const uint32_t nch = (j0 + n + 15) >> 4, end = j0 + n;  // end: bytes from ab
    auto ld = [&](uint32_t k) -> uint4 { return gload16(ab + 16ull * (k < nch ? k : 0)); };
    uint4 g0 = ld(0), g1 = ld(1), g2 = ld(2), g3 = ld(3);
    for (uint32_t k = 0; k < nch; k += 4) {
        const bool more = k + 4 < nch;
        uint4 h0 = g0, h1 = g1, h2 = g2, h3 = g3;
        if (more) { h0 = ld(k + 4); h1 = ld(k + 5); h2 = ld(k + 6); h3 = ld(k + 7); }
        auto one = [&](const uint4 &v, uint32_t kk) {
            if (kk >= nch) return;
            const uint32_t from = kk == 0 ? j0 : 0;
            const uint32_t to = 16 * kk + 16 <= end ? 16 : end - 16 * kk;
            c = crc_chunk_span(tabaddr, c, v, from, to - from);
        };
        one(g0, k);
        one(g1, k + 1);
        one(g2, k + 2);
        one(g3, k + 3);
        g0 = h0; g1 = h1; g2 = h2; g3 = h3;
    }
    return ~c;
}

// The same CRC with the bulk loads staged through LDS (kafka_classify): the
// next 64-byte batch is in flight into the wave's 4 KiB staging area (lane l's
// 16-byte pieces at 16 l of each 1 KiB block) while the current one is hashed
// from registers, so a lane's walk through a long message no longer waits a
// memory latency per batch -- the second buffer costs LDS, not VGPRs.  (cfg3:
// 0.929 -> 0.919 ms; holding the next batch in registers instead spills.)
// Correct under any exec mask: each active lane stages and reads only its own
// bytes, and a batch is waited for with vmcnt(0).  In pieces, so that the
// message-set walk can interleave them (read_message_set in kafka_classify).

// bytes before the first 16-byte boundary (at most 15, one chunk) in 8-, 4-
// and 1-byte steps; returns how many were hashed into c
__device__ __forceinline__ uint32_t crc_head(uint32_t tabaddr, Cur &cur, const uint8_t *p, uint32_t n, uint32_t &c) {
    uint32_t i = 0;
    const uint32_t k0 = (uint32_t)((uintptr_t)p & 15);
    uint32_t h = (16 - k0) & 15;
    if (h > n) h = n;
    if (h >= 4) {
        cur_fill(cur, (uintptr_t)p);
        if (h >= 8) {
            c = crc_step8(tabaddr, cur_word_at(cur, k0) ^ c, cur_word_at(cur, k0 + 4));
            i = 8;
        }
        if (h - i >= 4) {
            c = crc_step4(tabaddr, cur_word_at(cur, k0 + i) ^ c);
            i += 4;
        }
    }
    if (i < h) {
        cur_fill(cur, (uintptr_t)p);
        c = crc_bytes3(tabaddr, c, cur_word_at(cur, k0 + i), h - i);
        i = h;
    }
    return i;
}
// the 64 bytes at q (16-byte aligned) into the lane's staging slot
__device__ __forceinline__ void crc_stage(uint8_t *stage, const uint8_t *q) {
#pragma unroll
    for (int k = 0; k < 4; k++)
        __builtin_amdgcn_global_load_lds((const void *)(q + 16 * k),
                                         (__attribute__((address_space(3))) void *)(stage + k * 1024), 16, 0, 0);
}
// one staged 64-byte batch hashed into c; the next one (if any) staged meanwhile
__device__ __forceinline__ uint32_t crc_batch(const uint32_t *tab, uint8_t *stage, uint32_t c, const uint8_t *next) {
    const uint32_t la = (uint32_t)(uintptr_t)(stage + 16 * (threadIdx.x & 63));
    uint4 v0, v1, v2, v3;
    asm volatile("s_waitcnt vmcnt(0)\n\t"
                 "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                 "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
                 : "v"(la)
                 : "memory");
    if (next) crc_stage(stage, next);
#if L7G_KAFKA_CRCSTREAMS == 1
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint4 x = j < 2 ? v0 : j < 4 ? v1 : j < 6 ? v2 : v3;
        const uint32_t lo = ((j & 1) ? x.z : x.x) ^ c, hi = (j & 1) ? x.w : x.y;
        c = crc_slice8(tab, lo, hi);
    }
#elif L7G_KAFKA_CRCSTREAMS == 2
    // two independent chains (bytes 0-31 from c, bytes 32-63 from 0), joined
    // by the 32-zero-byte shift: 5 dependent lookup rounds, not 8
    uint32_t ca = c, cb = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        const uint4 xa = j < 2 ? v0 : v1, xb = j < 2 ? v2 : v3;
        ca = crc_slice8(tab, ((j & 1) ? xa.z : xa.x) ^ ca, (j & 1) ? xa.w : xa.y);
        cb = crc_slice8(tab, ((j & 1) ? xb.z : xb.x) ^ cb, (j & 1) ? xb.w : xb.y);
    }
    c = crc_shift(tab + kCrcZ32, ca) ^ cb;
#else
    // four chains of 16 bytes, joined by the 48/32/16-zero-byte shifts: 3 rounds
    uint32_t c0 = c, c1 = 0, c2 = 0, c3 = 0;
#pragma unroll
    for (int j = 0; j < 2; j++) {
        c0 = crc_slice8(tab, (j ? v0.z : v0.x) ^ c0, j ? v0.w : v0.y);
        c1 = crc_slice8(tab, (j ? v1.z : v1.x) ^ c1, j ? v1.w : v1.y);
        c2 = crc_slice8(tab, (j ? v2.z : v2.x) ^ c2, j ? v2.w : v2.y);
        c3 = crc_slice8(tab, (j ? v3.z : v3.x) ^ c3, j ? v3.w : v3.y);
    }
    c = crc_shift(tab + kCrcZ48, c0) ^ crc_shift(tab + kCrcZ32, c1) ^ crc_shift(tab + kCrcZ16, c2) ^ c3;
#endif
    return c;
}
// the rest (fewer than 64 bytes, from i, 16-byte aligned) from the cursor's
// chunks: 8-byte steps, then one 4-byte step, then bytes
__device__ __forceinline__ uint32_t crc_tail(uint32_t tabaddr, Cur &cur, const uint8_t *p, uint32_t n, uint32_t i,
                                             uint32_t c) {
    for (; i + 8 <= n; i += 8) {
        const uintptr_t a = (uintptr_t)(p + i);
        cur_fill(cur, a);
        const uint32_t k = (uint32_t)(a & 15);
        const uint32_t w0 = cur.w0, w1 = cur.w1, w2 = cur.w2, w3 = cur.w3;
        c = crc_step8(tabaddr, (k ? w2 : w0) ^ c, k ? w3 : w1);
    }
    if (i + 4 <= n) {
        const uintptr_t a = (uintptr_t)(p + i);
        cur_fill(cur, a);
        c = crc_step4(tabaddr, cur_word_at(cur, (uint32_t)(a & 15)) ^ c);
        i += 4;
    }
    if (i < n) {
        const uintptr_t a = (uintptr_t)(p + i);
        cur_fill(cur, a);
        c = crc_bytes3(tabaddr, c, cur_word_at(cur, (uint32_t)(a & 15)), n - i);
    }
    return c;
}
__device__ __forceinline__ uint32_t crc32_ieee_staged(const uint32_t *tab, Cur &cur, const uint8_t *p, uint32_t n,
                                                      uint8_t *stage) {
    const uint32_t tabaddr = (uint32_t)(uintptr_t)tab;
    uint32_t c = 0xFFFFFFFFu;
    uint32_t i = crc_head(tabaddr, cur, p, n, c);
    if (i + 64 <= n) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        crc_stage(stage, p + i);
        for (;;) {
            const bool more = i + 128 <= n;
            c = crc_batch(tab, stage, c, more ? p + i + 64 : nullptr);
            i += 64;
            if (!more) break;
        }
    }
    return ~crc_tail(tabaddr, cur, p, n, i, c);
}

}  // namespace
}  // namespace l7
