// Compressed Kafka message sets on gfx950 (product code).
//
// readMessageSet (vendor/github.com/optiopay/kafka/proto/messages.go:460-489)
// gunzips (codec 1: Go 1.10 compress/gzip + compress/flate) or snappy-decodes
// (codec 2: vendor/github.com/golang/snappy decode.go:25-73 with the xerial
// framing of proto/snappy.go:21-50) a message's value and reads the result as
// a message set, recursively; any decode error fails the whole request.  The
// verdict never depends on the inner messages' contents, only on whether they
// decode, so kafka_classify_kernel walks a request with compressed messages to
// its verdict as if they were plain (their key / value fields are still read)
// and lists it; this kernel then re-walks each listed request and decodes.
//
// One wave per listed request; lane 0 runs the sequential decoders (DEFLATE
// and snappy are serial bit / tag streams):
//   - the last 64 KiB of output live in an LDS ring, so back-references
//     (DEFLATE <= 32 KiB, snappy usually < 64 KiB) are served from LDS; longer
//     snappy offsets read the output already stored to HBM;
//   - output goes to the workgroup's slice of a decode region in HBM, one
//     dword store per 4 bytes, as a stack: a nested compressed message is
//     decoded above its parent's buffer and popped when its set ends;
//   - inner sets are walked from HBM with the same chunk cursor and slicing-
//     by-8 CRC as the classifier.
// Result per listed request: unchanged (every level decoded and parsed),
// PARSE_ERROR (a decode or inner-set error, as in the reference), or
// UNSUPPORTED when one nesting path needs more decoded bytes than the
// workgroup's region slice (out of contract; documented in DESIGN.md).
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "kafka_dec.h"

namespace l7 {

namespace {

constexpr uint32_t kWin = 65536;  // LDS history ring (power of two)
constexpr int kDepth = 8;         // nesting levels per request (beyond: UNSUPPORTED)

__constant__ uint16_t kLBase[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                    31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t kDBase[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,   33,   49,    65,    97,    129,
                                    193, 257, 385, 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

// canonical Huffman code (counts per length, symbols in code order)
struct Huff {
    uint16_t count[16];
    uint16_t sym[288];
};

// LDS of one workgroup (one wave)
struct ZShared {
    uint32_t crctab[kCrcSlices * 256];
    uint8_t win[kWin];
    Huff lit, dist, clen;
    uint8_t lens[320];
    uint16_t offs[16];
};

// Decoder output: a region buffer in HBM plus the LDS history ring.
struct ZOut {
    uint8_t *out;
    uint32_t cnt, cap;   // bytes written; the limit (kMaxParseBuf or what the region holds)
    uint32_t base;       // where the current gzip member / snappy block began
    uint32_t word;       // pending bytes of the dword being filled
    uint32_t crc;        // running CRC32 (gzip members)
    ZShared *sh;
};
__device__ __forceinline__ bool zput(ZOut &o, uint32_t b) {
    if (o.cnt >= o.cap) return false;
    const uint32_t k = o.cnt & 3;
    o.word = k ? o.word | (b << (8 * k)) : b;
    o.sh->win[o.cnt & (kWin - 1)] = (uint8_t)b;
    o.crc = o.sh->crctab[(o.crc ^ b) & 0xFF] ^ (o.crc >> 8);
    if (k == 3) *reinterpret_cast<uint32_t *>(o.out + o.cnt - 3) = o.word;
    o.cnt++;
    return true;
}
__device__ __forceinline__ void zflush(ZOut &o) {
    const uint32_t k = o.cnt & 3;  // the region slice has slack past cap for this dword
    if (k) *reinterpret_cast<uint32_t *>(o.out + o.cnt - k) = o.word;
}
// the byte `dist` (1 <= dist <= cnt) before the current position
__device__ __forceinline__ uint32_t zback(const ZOut &o, uint32_t dist) {
    if (dist <= kWin) return o.sh->win[(o.cnt - dist) & (kWin - 1)];
    return o.out[o.cnt - dist];  // >= 64 KiB back: already stored as a whole dword
}

// Compressed input: bytes [0, n) at p, LSB-first bit reader for DEFLATE.
struct ZIn {
    const uint8_t *p;
    uint32_t n, pos;
    uint32_t bits;
    int cnt;
    Cur cur;
};
__device__ __forceinline__ uint32_t zbyte(ZIn &s, uint32_t i) { return cur_byte(s.cur, s.p + i); }
__device__ __forceinline__ void zfill(ZIn &s) {
    while (s.cnt <= 24 && s.pos < s.n) {
        s.bits |= zbyte(s, s.pos++) << s.cnt;
        s.cnt += 8;
    }
}
__device__ __forceinline__ bool zbits(ZIn &s, int k, uint32_t &v) {
    if (s.cnt < k) {
        zfill(s);
        if (s.cnt < k) return false;
    }
    v = s.bits & ((1u << k) - 1u);
    s.bits = k == 32 ? 0 : s.bits >> k;
    s.cnt -= k;
    return true;
}
// to the next byte boundary; the bytes buffered but not used go back
__device__ __forceinline__ void zalign(ZIn &s) {
    s.pos -= (uint32_t)s.cnt >> 3;
    s.bits = 0;
    s.cnt = 0;
}

// huffmanDecoder.init (compress/flate/inflate.go): false for an over-
// subscribed or incomplete code, except the empty code and one code of length
// 1 (decoding then fails where a missing code is used).
__device__ bool hinit(Huff *h, uint16_t *offs, const uint8_t *len, int n) {
    for (int l = 0; l < 16; l++) h->count[l] = 0;
    int max = 0;
    for (int i = 0; i < n; i++) {
        h->count[len[i]]++;
        max = len[i] > max ? len[i] : max;
    }
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (uint16_t)(offs[l] + h->count[l]);
    for (int i = 0; i < n; i++)
        if (len[i]) h->sym[offs[len[i]]++] = (uint16_t)i;
    if (max == 0) return true;
    int64_t go = 0;
    for (int l = 1; l <= max; l++) go = (go << 1) + h->count[l];
    return go == (int64_t(1) << max) || (go == 1 && max == 1);
}
// one symbol, code bits MSB first; -1 end of input, -2 no such code
__device__ int hdecode(ZIn &s, const Huff *h) {
    if (s.cnt < 15) zfill(s);
    const uint32_t bits = s.bits;
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
        if (l > s.cnt) return -1;
        code |= (int)((bits >> (l - 1)) & 1u);
        const int count = h->count[l];
        if (code - count < first) {
            s.bits >>= l;
            s.cnt -= l;
            return h->sym[index + (code - first)];
        }
        index += count;
        first = (first + count) << 1;
        code <<= 1;
    }
    return -2;
}

// huffmanBlock: 0 end of block, -1 corrupt / short input, -3 output cap
__device__ int zcodes(ZIn &s, ZOut &o, const Huff *lit, const Huff *dist, bool fixed) {
    for (;;) {
        int sym = hdecode(s, lit);
        if (sym < 0) return -1;
        if (sym < 256) {
            if (!zput(o, (uint32_t)sym)) return -3;
            continue;
        }
        if (sym == 256) return 0;
        sym -= 257;
        if (sym >= 29) return -1;
        uint32_t e;
        if (!zbits(s, kLExt[sym], e)) return -1;
        const uint32_t len = kLBase[sym] + e;
        int ds;
        if (fixed) {
            uint32_t r;
            if (!zbits(s, 5, r)) return -1;
            ds = (int)(__builtin_bitreverse32(r) >> 27);  // 5 bits, most significant first
        } else {
            ds = hdecode(s, dist);
            if (ds < 0) return -1;
        }
        if (ds >= 30) return -1;
        if (!zbits(s, kDExt[ds], e)) return -1;
        const uint32_t d = kDBase[ds] + e;
        if (d > o.cnt - o.base) return -1;  // before this member's output
        for (uint32_t i = 0; i < len; i++)
            if (!zput(o, zback(o, d))) return -3;
    }
}

// one DEFLATE stream from s.pos (byte aligned); afterwards s.pos is the byte
// after the last bit used
__device__ int zinflate(ZIn &s, ZOut &o) {
    ZShared *sh = o.sh;
    s.bits = 0;
    s.cnt = 0;
    for (;;) {
        uint32_t fin, type;
        if (!zbits(s, 1, fin) || !zbits(s, 2, type)) return -1;
        int e = -1;
        if (type == 0) {  // stored
            zalign(s);
            if (s.pos + 4 > s.n) return -1;
            const uint32_t len = zbyte(s, s.pos) | zbyte(s, s.pos + 1) << 8;
            const uint32_t nlen = zbyte(s, s.pos + 2) | zbyte(s, s.pos + 3) << 8;
            s.pos += 4;
            if (len != (~nlen & 0xFFFFu)) return -1;
            if (s.pos + len > s.n) return -1;
            for (uint32_t i = 0; i < len; i++)
                if (!zput(o, zbyte(s, s.pos + i))) return -3;
            s.pos += len;
            e = 0;
        } else if (type == 1) {  // fixed codes
            for (int i = 0; i < 144; i++) sh->lens[i] = 8;
            for (int i = 144; i < 256; i++) sh->lens[i] = 9;
            for (int i = 256; i < 280; i++) sh->lens[i] = 7;
            for (int i = 280; i < 288; i++) sh->lens[i] = 8;
            hinit(&sh->lit, sh->offs, sh->lens, 288);
            e = zcodes(s, o, &sh->lit, nullptr, true);
        } else if (type == 2) {  // dynamic codes (readHuffman)
            uint32_t v;
            if (!zbits(s, 5, v)) return -1;
            const int nlit = (int)v + 257;
            if (!zbits(s, 5, v)) return -1;
            const int ndist = (int)v + 1;
            if (!zbits(s, 4, v)) return -1;
            const int nclen = (int)v + 4;
            if (nlit > 286 || ndist > 30) return -1;
            uint8_t *cl = sh->lens + 288;  // 19 code-length code lengths (lens[288..307))
            for (int i = 0; i < 19; i++) cl[i] = 0;
            for (int i = 0; i < nclen; i++) {
                if (!zbits(s, 3, v)) return -1;
                cl[kOrder[i]] = (uint8_t)v;
            }
            if (!hinit(&sh->clen, sh->offs, cl, 19)) return -1;
            // the lengths of both codes, lens[0, nlit + ndist): this may run into
            // cl, which is no longer needed once clen is built
            uint8_t *bits = sh->lens;
            const int total = nlit + ndist;
            for (int i = 0; i < total;) {
                const int sym = hdecode(s, &sh->clen);
                if (sym < 0) return -1;
                if (sym < 16) {
                    bits[i++] = (uint8_t)sym;
                    continue;
                }
                int rep, nb;
                uint8_t b;
                if (sym == 16) {
                    if (i == 0) return -1;
                    rep = 3; nb = 2; b = bits[i - 1];
                } else if (sym == 17) {
                    rep = 3; nb = 3; b = 0;
                } else {
                    rep = 11; nb = 7; b = 0;
                }
                if (!zbits(s, nb, v)) return -1;
                rep += (int)v;
                if (i + rep > total) return -1;
                while (rep--) bits[i++] = b;
            }
            if (!hinit(&sh->lit, sh->offs, bits, nlit) || !hinit(&sh->dist, sh->offs, bits + nlit, ndist)) return -1;
            e = zcodes(s, o, &sh->lit, &sh->dist, false);
        }
        if (e) return e;
        if (fin) break;
    }
    zalign(s);
    return 0;
}

__device__ uint32_t crc_bytes(const uint32_t *tab, uint32_t c, ZIn &s, uint32_t at, uint32_t n) {
    for (uint32_t i = 0; i < n; i++) c = tab[(c ^ zbyte(s, at + i)) & 0xFF] ^ (c >> 8);
    return c;
}

// gzip.NewReader + ioutil.ReadAll (gunzip.go: readHeader, multistream Read):
// 0 ok, -1 error, -3 output cap
__device__ int zgunzip(ZIn &s, ZOut &o) {
    const uint32_t *tab = o.sh->crctab;
    const uint32_t n = s.n;
    for (int member = 0;; member++) {
        if (s.pos == n) {
            if (member == 0) return -1;  // io.EOF from NewReader
            break;
        }
        if (n - s.pos < 10) return -1;
        const uint32_t h = s.pos;
        if (zbyte(s, h) != 0x1f || zbyte(s, h + 1) != 0x8b || zbyte(s, h + 2) != 8) return -1;
        const uint32_t flg = zbyte(s, h + 3);
        uint32_t digest = crc_bytes(tab, 0xFFFFFFFFu, s, h, 10);
        s.pos += 10;
        if (flg & 0x04) {  // FEXTRA
            if (n - s.pos < 2) return -1;
            const uint32_t xl = zbyte(s, s.pos) | zbyte(s, s.pos + 1) << 8;
            digest = crc_bytes(tab, digest, s, s.pos, 2);
            s.pos += 2;
            if (n - s.pos < xl) return -1;
            digest = crc_bytes(tab, digest, s, s.pos, xl);
            s.pos += xl;
        }
        for (uint32_t f = 0x08; f <= 0x10; f <<= 1) {  // FNAME, FCOMMENT: readString (512-byte buffer)
            if (!(flg & f)) continue;
            uint32_t i = 0;
            for (;; i++) {
                if (i >= 512) return -1;
                if (s.pos + i >= n) return -1;
                if (zbyte(s, s.pos + i) == 0) break;
            }
            digest = crc_bytes(tab, digest, s, s.pos, i + 1);
            s.pos += i + 1;
        }
        if (flg & 0x02) {  // FHCRC
            if (n - s.pos < 2) return -1;
            const uint32_t hc = zbyte(s, s.pos) | zbyte(s, s.pos + 1) << 8;
            if (hc != (~digest & 0xFFFFu)) return -1;
            s.pos += 2;
        }
        const uint32_t start = o.cnt;
        o.base = start;
        o.crc = 0xFFFFFFFFu;
        const int e = zinflate(s, o);
        if (e) return e;
        if (n - s.pos < 8) return -1;
        const uint32_t t = s.pos;
        const uint32_t crc = zbyte(s, t) | zbyte(s, t + 1) << 8 | zbyte(s, t + 2) << 16 | zbyte(s, t + 3) << 24;
        const uint32_t isz = zbyte(s, t + 4) | zbyte(s, t + 5) << 8 | zbyte(s, t + 6) << 16 | zbyte(s, t + 7) << 24;
        s.pos += 8;
        if (crc != ~o.crc || isz != o.cnt - start) return -1;
    }
    return 0;
}

// snappy.Decode of the block at [at, at + n) of s: 0 ok, -1 error, -3 output cap
__device__ int zsnappy_block(ZIn &s, uint32_t at, uint32_t n, ZOut &o) {
    uint64_t v = 0;
    uint32_t hl = 0;
    for (int sh = 0;; sh += 7) {  // decodedLen: binary.Uvarint
        if (hl >= n) return -1;
        const uint32_t b = zbyte(s, at + hl++);
        if (hl == 10 && b > 1) return -1;
        v |= (uint64_t)(b & 0x7F) << sh;
        if (b < 0x80) break;
        if (hl == 10) return -1;
    }
    if (v > 0xFFFFFFFFull) return -1;
    if (v > o.cap - o.cnt) return -3;
    const uint32_t dlen = (uint32_t)v;
    o.base = o.cnt;
    uint32_t i = hl;
    while (i < n) {
        const uint32_t d = o.cnt - o.base;
        const uint32_t tag = zbyte(s, at + i);
        uint32_t length, offset;
        const uint32_t kind = tag & 3;
        if (kind == 0) {  // literal
            uint32_t x = tag >> 2;
            if (x < 60) {
                i++;
            } else {
                const uint32_t k = x - 59;  // 1..4 length bytes
                i += 1 + k;
                if (i > n) return -1;
                x = 0;
                for (uint32_t j = 0; j < k; j++) x |= zbyte(s, at + i - k + j) << (8 * j);
            }
            const uint64_t llen = (uint64_t)x + 1;  // Go: int(x) + 1, 2^32 for x = 0xFFFFFFFF
            if (llen > dlen - d || llen > n - i) return -1;
            for (uint32_t j = 0; j < (uint32_t)llen; j++) zput(o, zbyte(s, at + i + j));
            i += (uint32_t)llen;
            continue;
        }
        if (kind == 1) {
            i += 2;
            if (i > n) return -1;
            const uint32_t t0 = zbyte(s, at + i - 2);
            length = 4 + ((t0 >> 2) & 7);
            offset = (t0 & 0xE0) << 3 | zbyte(s, at + i - 1);
        } else if (kind == 2) {
            i += 3;
            if (i > n) return -1;
            length = 1 + (zbyte(s, at + i - 3) >> 2);
            offset = zbyte(s, at + i - 2) | zbyte(s, at + i - 1) << 8;
        } else {
            i += 5;
            if (i > n) return -1;
            length = 1 + (zbyte(s, at + i - 5) >> 2);
            offset = zbyte(s, at + i - 4) | zbyte(s, at + i - 3) << 8 | zbyte(s, at + i - 2) << 16 |
                     zbyte(s, at + i - 1) << 24;
        }
        if (offset == 0 || d < offset || length > dlen - d) return -1;
        for (uint32_t j = 0; j < length; j++) zput(o, zback(o, offset));
    }
    if (o.cnt - o.base != dlen) return -1;
    return 0;
}

// snappyDecode (proto/snappy.go): plain snappy, or the xerial framing
__device__ int zunsnappy(ZIn &s, ZOut &o) {
    const uint32_t n = s.n;
    const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    bool xerial = n >= 8;
    for (int i = 0; i < 8 && xerial; i++) xerial = zbyte(s, i) == magic[i];
    if (!xerial) return zsnappy_block(s, 0, n, o);
    if (n < 12) return -1;  // b[8:12] out of range: a panic in the reference
    const uint32_t ver = zbyte(s, 8) << 24 | zbyte(s, 9) << 16 | zbyte(s, 10) << 8 | zbyte(s, 11);
    if (ver != 1) return -1;
    for (uint32_t i = 16; i < n;) {
        if (n - i < 4) return -1;
        const uint32_t cn = zbyte(s, i) << 24 | zbyte(s, i + 1) << 16 | zbyte(s, i + 2) << 8 | zbyte(s, i + 3);
        i += 4;
        if (cn > n - i) return -1;
        const int e = zsnappy_block(s, i, cn, o);
        if (e) return e;
        i += cn;
    }
    return 0;
}

struct ZCtx {
    ZShared *sh;
    uint8_t *region;       // this workgroup's slice
    uint32_t region_bytes;
    Cur cur;               // message-walk cursor
};

// readMessageSet over [pos, end) of b with every compressed message decoded
// and its set read recursively (explicit stack; each level's decoded bytes sit
// above its parent's in the region slice).  0 ok, -1 error (the request fails),
// -2 the region slice or the nesting stack is too small (UNSUPPORTED).
__device__ int zset(ZCtx &z, const uint8_t *b, uint32_t &pos, uint32_t end, int32_t size, int16_t version) {
    if (size < 0) return 0;
    if ((uint32_t)size > kMaxParseBuf) return -1;
    const uint8_t *fb[kDepth];
    uint32_t fpos[kDepth], fend[kDepth], fbuf[kDepth];
    int32_t flim[kDepth];  // LimitReader counts: at most the 16 MiB region slice
    int depth = 0;
    fb[0] = b; fpos[0] = pos; fend[0] = end; flim[0] = size; fbuf[0] = 0;
    uint32_t top = 0;  // first free byte of the region slice
    int rc = 0;
    for (;;) {
        const uint8_t *fbd = fb[depth];
        KDec dec{fbd, fpos[depth], fend[depth], flim[depth], 0, &z.cur};
        bool stop = false, push = false;
        uint32_t vat = 0, vlen = 0;
        int codec = 0;
        dec_skip(dec, 8);
        int32_t msize = 0;
        if (dec.err) stop = true;
        if (!stop) {
            msize = (int32_t)dec_int(dec, 4);
            if (dec.err || msize <= 0) stop = true;
        }
        if (!stop && (uint32_t)msize > kMaxParseBuf) { rc = -1; break; }
        uint32_t at = 0;
        if (!stop) {
            at = kread(dec, (uint32_t)msize);
            if (dec.err) stop = true;
        }
        if (!stop) {
            KDec md{fbd, at, at + (uint32_t)msize, -1, 0, &z.cur};
            const uint32_t crc = (uint32_t)dec_int(md, 4);
            if (msize <= 4 || crc != crc32_ieee(z.sh->crctab, z.cur, fbd + at + 4, (uint32_t)msize - 4)) {
                stop = true;  // stop, no drain
            } else {
                dec_skip(md, 1);
                const int8_t attr = (int8_t)dec_int(md, 1);
                if (version >= 1) dec_skip(md, 8);
                codec = attr & 3;
                if (codec == 3) {
                    stop = true;
                } else {
                    dec_bytes(md);
                    if (codec == 0) {
                        dec_bytes(md);
                    } else if (!md.err) {  // the value: where and how long
                        const int32_t sl = (int32_t)dec_int(md, 4);
                        if (!md.err && sl >= 1) {
                            if ((uint32_t)sl > kMaxParseBuf) md.err = 3;
                            else { vat = kread(md, (uint32_t)sl); if (!md.err) vlen = (uint32_t)sl; }
                        }
                    }
                    if (md.err) { rc = -1; break; }
                    push = codec != 0;
                }
            }
        }
        fpos[depth] = dec.pos;
        flim[depth] = dec.limit;
        if (stop) {
            if (depth == 0) break;
            top = fbuf[depth];
            depth--;
            continue;
        }
        if (!push) continue;
        if (depth + 1 == kDepth) { rc = -2; break; }
        // decode the value into the region slice above the parent's bytes
        const uint32_t room = top + 64 <= z.region_bytes ? z.region_bytes - top - 64 : 0;
        const bool region_bound = room < kMaxParseBuf;
        ZOut o{z.region + top, 0, region_bound ? room : kMaxParseBuf, 0, 0, 0xFFFFFFFFu, z.sh};
        ZIn s{fbd + vat, vlen, 0, 0, 0, {}};
        s.cur.line = ~(uintptr_t)0;
        const int e = codec == 1 ? zgunzip(s, o) : codec == 2 ? zunsnappy(s, o) : -1;
        if (e) { rc = (e == -3 && region_bound) ? -2 : -1; break; }
        zflush(o);
        z.cur.line = ~(uintptr_t)0;  // the slice may hold a popped level's bytes in the cursor
        depth++;
        fb[depth] = z.region + top;
        fpos[depth] = 0;
        fend[depth] = o.cnt;
        flim[depth] = o.cnt;
        fbuf[depth] = top;
        top += (o.cnt + 15u) & ~15u;
        top += 16;
    }
    pos = fpos[0];
    return rc;
}

// Re-walk a listed Produce request (its structure already parsed without
// error by kafka_classify_kernel) and decode its compressed messages.
__device__ int zrequest(ZCtx &z, const uint8_t *b) {
    Cur &cur = z.cur;
    const uint32_t rawlen = (uint32_t)be_load(cur, b, 4) + 4;
    KDec d{b, 0, rawlen, -1, 0, &cur};
    bool bad = false;
    dec_skip(d, 4); dec_skip(d, 2);
    const int16_t ver = (int16_t)dec_int(d, 2);
    dec_skip(d, 4);
    uint32_t o, l;
    dec_string(d, o, l);
    if (ver >= 3) dec_string(d, o, l);
    dec_skip(d, 2); dec_skip(d, 4);
    const int32_t nt = dec_arraylen(d, false, bad);
    if (bad || d.err) return 0;
    for (int32_t t = 0; t < nt; t++) {
        dec_string(d, o, l);
        if (d.err) return 0;
        const int32_t np = dec_arraylen(d, false, bad);
        if (bad) return 0;
        for (int32_t p = 0; p < np; p++) {
            dec_skip(d, 4);
            if (d.err) return 0;
            const int32_t ss = (int32_t)dec_int(d, 4);
            if (d.err) return 0;
            const int rc = zset(z, b, d.pos, d.end, ss, ver);
            if (rc) return rc;
        }
    }
    return 0;
}

}  // namespace

__global__ __launch_bounds__(64) void kafka_inflate_kernel(Batch B, const uint32_t *__restrict__ zlist,
                                                           const uint32_t *__restrict__ zcount, uint8_t *region,
                                                           uint32_t region_bytes) {
    __shared__ ZShared sh;
    const uint32_t count = *zcount;
    if (blockIdx.x >= count) return;
    {  // CRC tables, 4 entries per lane
        for (uint32_t t = threadIdx.x; t < 256; t += 64) {
            uint32_t c = t;
            for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
            sh.crctab[t] = c;
        }
        __syncthreads();
        for (int k = 1; k < kCrcSlices; k++) {
            for (uint32_t t = threadIdx.x; t < 256; t += 64) {
                const uint32_t prev = sh.crctab[(k - 1) * 256 + t];
                sh.crctab[k * 256 + t] = (prev >> 8) ^ sh.crctab[prev & 0xFF];
            }
            __syncthreads();
        }
    }
    if (threadIdx.x != 0) return;
    ZCtx z;
    z.sh = &sh;
    z.region = region + (size_t)blockIdx.x * region_bytes;
    z.region_bytes = region_bytes;
    for (uint32_t k = blockIdx.x; k < count; k += gridDim.x) {
        const uint32_t idx = zlist[k];
        z.cur.line = ~(uintptr_t)0;
        const int rc = zrequest(z, B.arena + B.offs[idx]);
        if (rc) {
            B.verdict[idx] = rc == -1 ? V_PARSE_ERROR : V_UNSUPPORTED;
            B.rule[idx] = -1;
            B.consumed[idx] = 0;
        }
    }
}

uint32_t KafkaInflateBlocks() { return 64; }
uint32_t KafkaInflateRegionBytes() { return 16u << 20; }

hipError_t LaunchKafkaInflate(const Batch &B, const uint32_t *zlist, const uint32_t *zcount, uint8_t *region,
                              hipStream_t stream) {
    if (B.n == 0) return hipSuccess;
    hipLaunchKernelGGL(kafka_inflate_kernel, dim3(KafkaInflateBlocks()), dim3(64), 0, stream, B, zlist, zcount, region,
                       KafkaInflateRegionBytes());
    return hipGetLastError();
}

}  // namespace l7
