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
constexpr int kCrcTables = 8;  // slicing-by-8: T_k[b] = the register after byte b and k zero bytes
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
        for (int k = 1; k < kCrcTables; k++) {
            v = (v >> 8) ^ tab[v & 0xFF];  // T_k[t]
            tab[k * 256 + t] = v;
        }
    }
    __syncthreads();
}
__device__ __forceinline__ uint32_t crc_slice8(const uint32_t *tab, uint32_t lo, uint32_t hi) {
    return tab[7 * 256 + (lo & 0xFF)] ^ tab[6 * 256 + ((lo >> 8) & 0xFF)] ^ tab[5 * 256 + ((lo >> 16) & 0xFF)] ^
           tab[4 * 256 + (lo >> 24)] ^ tab[3 * 256 + (hi & 0xFF)] ^ tab[2 * 256 + ((hi >> 8) & 0xFF)] ^
           tab[1 * 256 + ((hi >> 16) & 0xFF)] ^ tab[hi >> 24];
}
constexpr uint32_t kInf = 0xFFFFFFFFu;

// Per-lane byte cursor: the decoders walk their request forward, so each lane
// keeps the 16-byte aligned chunk it last touched in registers and serves
// field bytes from it; one dwordx4 load replaces up to 16 byte loads.  A chunk
// that holds a request byte never leaves that byte's page, so the aligned
// over-read is safe for any arena alignment.
struct Cur {
    uintptr_t line;  // address of the cached chunk (~0 = none)
    uint32_t w0, w1, w2, w3;  // scalars, not an array: a selected array element would put Cur in scratch
};
__device__ __forceinline__ void cur_fill(Cur &c, uintptr_t a) {
    const uintptr_t ln = a & ~(uintptr_t)15;
    if (ln != c.line) {
        const uint4 v = gload16(ln);
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

struct KDec {
    const uint8_t *b;
    uint32_t pos, end;
    int32_t limit;  // LimitReader remaining, -1 = none (a set is at most kMaxParseBuf)
    int err;        // 0 ok, 1 EOF, 2 ErrUnexpectedEOF, 3 other
    Cur *c;
};

__device__ __forceinline__ uint32_t kavail(const KDec &d) {
    uint32_t a = d.end - d.pos;
    if (d.limit >= 0 && (uint32_t)d.limit < a) a = (uint32_t)d.limit;
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
    if (d.limit >= 0) d.limit -= (int32_t)take;
    if (take < n) d.err = 2;
    return at;
}
// Big-endian n-byte field (n = 1, 2, 4 or 8).  A field inside the cached
// 16-byte chunk is cut out of two adjacent words (v_alignbyte) and byte-
// swapped (v_perm); one straddling two chunks is read byte by byte.
__device__ __forceinline__ uint32_t bswap32(uint32_t x) { return __builtin_amdgcn_perm(0, x, 0x00010203u); }
__device__ __forceinline__ uint64_t be_load(Cur &c, const uint8_t *p, int n) {
    const uintptr_t a = (uintptr_t)p;
    const uint32_t k = (uint32_t)(a & 15);
    if (n <= 4 && k + (uint32_t)n <= 16) {
        cur_fill(c, a);
        const uint32_t w0 = c.w0, w1 = c.w1, w2 = c.w2, w3 = c.w3;
        const uint32_t i = k >> 2;
        const uint32_t lo = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
        const uint32_t hi = i == 0 ? w1 : i == 1 ? w2 : i == 2 ? w3 : 0u;
        const uint32_t v = bswap32(__builtin_amdgcn_alignbyte(hi, lo, k & 3));  // bytes k..k+3, big-endian
        return n == 4 ? v : v >> (32 - 8 * n);
    }
    if (n == 8) return (be_load(c, p, 4) << 32) | be_load(c, p + 4, 4);
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | cur_byte(c, p + i);
    return v;
}
__device__ __forceinline__ int64_t dec_int(KDec &d, int n) {
    if (d.err) return 0;
    uint32_t at = kread(d, (uint32_t)n);
    if (d.err) return 0;
    uint64_t v = be_load(*d.c, d.b + at, n);
    return n == 1 ? (int64_t)(int8_t)v : n == 2 ? (int64_t)(int16_t)v : n == 4 ? (int64_t)(int32_t)v : (int64_t)v;
}
// A field whose value is not needed: only the read (and its errors) matter.
__device__ __forceinline__ void dec_skip(KDec &d, int n) {
    if (d.err) return;
    kread(d, (uint32_t)n);
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
__device__ __forceinline__ int32_t dec_arraylen(KDec &d, bool nullable, bool &bad) {
    int32_t l = (int32_t)dec_int(d, 4);
    bad = false;
    if (l < 0) { if (nullable) return -1; bad = true; return 0; }
    if ((uint32_t)l > kMaxParseBuf) { bad = true; return 0; }
    return l;
}
__device__ __forceinline__ void dec_bytes(KDec &d) {
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

// The same CRC with the bulk loads staged through LDS (kafka_classify): the
// next 64-byte batch is in flight into the wave's 4 KiB staging area (lane l's
// 16-byte pieces at 16 l of each 1 KiB block) while the current one is hashed
// from registers, so a lane's walk through a long message no longer waits a
// memory latency per batch -- the second buffer costs LDS, not VGPRs.  (cfg3:
// 0.929 -> 0.919 ms; holding the next batch in registers instead spills.)
// Correct under any exec mask: each active lane stages and reads only its own
// bytes, and a batch is waited for with vmcnt(0).  The last, short batch is
// staged too (crc_last): its up to four chunks cost one round trip, where the
// cursor took one per chunk (cfg5 Kafka 16.45 -> 16.10 ms).  A message the walk
// reads through its window starts from the window already in the slot
// (crc32_ieee_window).

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
// the 64 bytes at q (16-byte aligned) into the lane's staging slot, chunks
// past lastc (the request's last one) clamped to it: a message's last batch
// is staged like the others and only its own bytes are read back
__device__ __forceinline__ void crc_stage(uint8_t *stage, const uint8_t *q, uintptr_t lastc) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const uintptr_t a = (uintptr_t)(q + 16 * k);
        __builtin_amdgcn_global_load_lds((const void *)(k == 0 || a <= lastc ? a : lastc),
                                         (__attribute__((address_space(3))) void *)(stage + k * 1024), 16, 0, 0);
    }
}
// one staged 64-byte batch hashed into c; the next one (if any) staged meanwhile
__device__ __forceinline__ uint32_t crc_batch(const uint32_t *tab, uint8_t *stage, uint32_t c, const uint8_t *next,
                                              uintptr_t lastc) {
    const uint32_t la = (uint32_t)(uintptr_t)(stage + 16 * (threadIdx.x & 63));
    uint4 v0, v1, v2, v3;
    asm volatile("s_waitcnt vmcnt(0)\n\t"
                 "ds_read_b128 %0, %4\n\tds_read_b128 %1, %4 offset:1024\n\t"
                 "ds_read_b128 %2, %4 offset:2048\n\tds_read_b128 %3, %4 offset:3072\n\t"
                 "s_waitcnt lgkmcnt(0)"
                 : "=v"(v0), "=v"(v1), "=v"(v2), "=v"(v3)
                 : "v"(la)
                 : "memory");
    if (next) crc_stage(stage, next, lastc);
#pragma unroll
    for (int j = 0; j < 8; j++) {
        const uint4 x = j < 2 ? v0 : j < 4 ? v1 : j < 6 ? v2 : v3;
        const uint32_t lo = ((j & 1) ? x.z : x.x) ^ c, hi = (j & 1) ? x.w : x.y;
        c = crc_slice8(tab, lo, hi);
    }
    return c;
}
// the staged last batch's rem (1 .. 63) bytes: 8-byte steps, then one
// 4-byte step, then bytes, each word read back from the lane's staging slot
__device__ __forceinline__ uint32_t lds_word_at(uint32_t la, uint32_t j) {  // bytes j .. j+3 (j % 4 == 0)
    uint32_t x;
    asm volatile("ds_read_b32 %0, %1\n\ts_waitcnt lgkmcnt(0)" : "=v"(x) : "v"(la + ((j >> 4) << 10) + (j & 15)) : "memory");
    return x;
}
// (bytes [j0, rem) of the slot: j0 a multiple of 8)
__device__ __forceinline__ uint32_t crc_last(uint32_t tabaddr, uint8_t *stage, uint32_t rem, uint32_t c,
                                             uint32_t j0 = 0) {
    const uint32_t la = (uint32_t)(uintptr_t)(stage + 16 * (threadIdx.x & 63));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    uint32_t j = j0;
    for (; j + 8 <= rem; j += 8) {
        uint64_t x;
        asm volatile("ds_read_b64 %0, %1\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(x)
                     : "v"(la + ((j >> 4) << 10) + (j & 8))
                     : "memory");
        c = crc_step8(tabaddr, (uint32_t)x ^ c, (uint32_t)(x >> 32));
    }
    if (j + 4 <= rem) {
        c = crc_step4(tabaddr, lds_word_at(la, j) ^ c);
        j += 4;
    }
    if (j < rem) c = crc_bytes3(tabaddr, c, lds_word_at(la, j), rem - j);
    return c;
}
// Every byte after the head (crc_head) comes through the staging slot, the
// last (short) batch included: a message's bytes cost one memory round trip
// per 64, the next batch in flight while one is hashed.
__device__ __forceinline__ uint32_t crc32_ieee_staged(const uint32_t *tab, Cur &cur, const uint8_t *p, uint32_t n,
                                                      uint8_t *stage, uintptr_t lastc) {
    const uint32_t tabaddr = (uint32_t)(uintptr_t)tab;
    uint32_t c = 0xFFFFFFFFu;
    uint32_t i = crc_head(tabaddr, cur, p, n, c);
    if (i < n) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        crc_stage(stage, p + i, lastc);
        while (i + 64 <= n) {
            const bool more = i + 64 < n;
            c = crc_batch(tab, stage, c, more ? p + i + 64 : nullptr, lastc);
            i += 64;
        }
        if (i < n) c = crc_last(tabaddr, stage, n - i, c);
    }
    return ~c;
}
// The same CRC for a message whose 64-byte window [c0, c0 + 64) the walk has
// just staged into the slot (c0 = the chunk of the message's offset field,
// p - 16): the CRC's bytes up to c0 + 64 are hashed from the slot, and the
// first batch from memory is c0 + 64's, staged while they are hashed.
__device__ __forceinline__ uint32_t crc32_ieee_window(const uint32_t *tab, Cur &cur, const uint8_t *p, uint32_t n,
                                                      uint8_t *stage, uintptr_t lastc) {
    const uint32_t tabaddr = (uint32_t)(uintptr_t)tab;
    uint32_t c = 0xFFFFFFFFu;
    uint32_t i = crc_head(tabaddr, cur, p, n, c);
    if (i < n) {
        const uint8_t *c0 = reinterpret_cast<const uint8_t *>((uintptr_t)(p - 16) & ~(uintptr_t)15);
        const uint32_t o = (uint32_t)((p + i) - c0);  // 16 or 32
        if (n - i <= 64 - o) return ~crc_last(tabaddr, stage, o + (n - i), c, o);
        const uint32_t la = (uint32_t)(uintptr_t)(stage + 16 * (threadIdx.x & 63));
        uint4 v1, v2, v3;
        asm volatile("ds_read_b128 %0, %3 offset:1024\n\tds_read_b128 %1, %3 offset:2048\n\t"
                     "ds_read_b128 %2, %3 offset:3072\n\ts_waitcnt lgkmcnt(0)"
                     : "=v"(v1), "=v"(v2), "=v"(v3)
                     : "v"(la)
                     : "memory");
        crc_stage(stage, c0 + 64, lastc);
        const uint32_t j0 = o == 16 ? 0 : 2;
#pragma unroll
        for (uint32_t j = 0; j < 6; j++) {
            if (j < j0) continue;
            const uint4 x = j < 2 ? v1 : j < 4 ? v2 : v3;
            const uint32_t lo = ((j & 1) ? x.z : x.x) ^ c, hi = (j & 1) ? x.w : x.y;
            c = crc_slice8(tab, lo, hi);
        }
        i += 64 - o;
        while (i + 64 <= n) {
            const bool more = i + 64 < n;
            c = crc_batch(tab, stage, c, more ? p + i + 64 : nullptr, lastc);
            i += 64;
        }
        if (i < n) c = crc_last(tabaddr, stage, n - i, c);
    }
    return ~c;
}

}  // namespace
}  // namespace l7
