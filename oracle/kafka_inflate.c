/*
 * kafka_inflate.c — TEST INFRASTRUCTURE ONLY (parity oracle, see l7ref.h).
 *
 * The decoders readMessageSet calls for a compressed message
 * (vendor/github.com/optiopay/kafka/proto/messages.go:460-489), restated:
 *
 *   gzip: Go 1.10 compress/gzip Reader (gunzip.go: readHeader, Read with
 *         multistream) over compress/flate (inflate.go: nextBlock,
 *         readHuffman, huffmanBlock, dataBlock; huffmanDecoder.init).  Go 1.10
 *         is the toolchain the reference pins (envoy/Dockerfile:19); the
 *         stdlib is not vendored, so this follows its published algorithm.
 *   snappy: vendor/github.com/golang/snappy/decode.go:25-73 (decodedLen,
 *         Decode) and decode_other.go (decode), plus the xerial framing of
 *         vendor/github.com/optiopay/kafka/proto/snappy.go:21-50.
 *
 * Only success / failure and the decoded bytes matter to the verdict (any
 * error makes ReadProduceReq fail).  Output is capped at `cap` bytes: a larger
 * result fails readMessageSet's size check (messages.go:369-371) whatever
 * else happens, so decoding stops there.  Where Go would panic (a xerial
 * stream cut inside its header or a chunk) the result is an error.
 */
#include <stdlib.h>
#include <string.h>
#include "ref_internal.h"

/* ------------------------------------------------------------ flate */
typedef struct {
    const uint8_t *in; size_t n, pos;
    uint32_t bitbuf; int bitcnt;
    uint8_t *out; size_t cap, cnt;
    size_t base;  /* output position where the current member began */
} inf_t;

/* next bit (LSB first, bytes read as needed); -1 at end of input */
static int inf_bit(inf_t *s) {
    if (s->bitcnt == 0) {
        if (s->pos >= s->n) return -1;
        s->bitbuf = s->in[s->pos++];
        s->bitcnt = 8;
    }
    int b = (int)(s->bitbuf & 1);
    s->bitbuf >>= 1;
    s->bitcnt--;
    return b;
}
static int inf_bits(inf_t *s, int k, uint32_t *v) {
    uint32_t x = 0;
    for (int i = 0; i < k; i++) {
        int b = inf_bit(s);
        if (b < 0) return -1;
        x |= (uint32_t)b << i;
    }
    *v = x;
    return 0;
}

typedef struct { short count[16]; short symbol[288]; } huff_t;

/* huffmanDecoder.init: false for an over-subscribed or incomplete code,
 * except the empty code and a single code of length 1 (accepted; decoding
 * with them fails where the missing codes are used) */
static int huff_init(huff_t *h, const short *len, int n) {
    memset(h->count, 0, sizeof h->count);
    int max = 0;
    for (int i = 0; i < n; i++) { h->count[len[i]]++; if (len[i] > max) max = len[i]; }
    short offs[16];
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = (short)(offs[l] + h->count[l]);
    for (int i = 0; i < n; i++) if (len[i]) h->symbol[offs[len[i]]++] = (short)i;
    if (max == 0) return 1;
    long go = 0;  /* sum of count[l] * 2^(max-l): 2^max for a complete code */
    int min = 0;
    for (int l = 1; l <= max; l++) if (h->count[l]) { min = l; break; }
    for (int l = min; l <= max; l++) go = (go << 1) + h->count[l];
    if (go != (1L << max) && !(go == 1 && max == 1)) return 0;
    return 1;
}
/* canonical decode, one bit at a time; -1 end of input, -2 no such code */
static int huff_decode(inf_t *s, const huff_t *h) {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
        int b = inf_bit(s);
        if (b < 0) return -1;
        code |= b;
        int count = h->count[l];
        if (code - count < first) return h->symbol[index + (code - first)];
        index += count;
        first += count;
        first <<= 1;
        code <<= 1;
    }
    return -2;
}

static const short kLBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const short kLExt[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const short kDBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385,
                                 513, 769, 1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const short kDExt[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

static int inf_put(inf_t *s, uint8_t b) {
    if (s->cnt >= s->cap) return -1;
    s->out[s->cnt++] = b;
    return 0;
}

/* huffmanBlock: symbols until end of block */
static int inf_codes(inf_t *s, const huff_t *lit, const huff_t *dist, int fixed_dist) {
    for (;;) {
        int sym = huff_decode(s, lit);
        if (sym < 0) return -1;
        if (sym < 256) { if (inf_put(s, (uint8_t)sym)) return -1; continue; }
        if (sym == 256) return 0;
        sym -= 257;
        if (sym >= 29) return -1;  /* 286, 287 */
        uint32_t e;
        if (inf_bits(s, kLExt[sym], &e)) return -1;
        int len = kLBase[sym] + (int)e;
        int ds;
        if (fixed_dist) {  /* 5 bits, most significant first */
            uint32_t r = 0;
            for (int i = 0; i < 5; i++) { int b = inf_bit(s); if (b < 0) return -1; r = (r << 1) | (uint32_t)b; }
            ds = (int)r;
        } else {
            ds = huff_decode(s, dist);
            if (ds < 0) return -1;
        }
        if (ds >= 30) return -1;
        if (inf_bits(s, kDExt[ds], &e)) return -1;
        size_t d = (size_t)kDBase[ds] + e;
        /* before the start of this member's output: each gzip member gets a
         * fresh flate reader (gunzip.go readHeader: Reset(z.r, nil)), so its
         * history never reaches into the previous member */
        if (d > s->cnt - s->base) return -1;
        for (int i = 0; i < len; i++) if (inf_put(s, s->out[s->cnt - d])) return -1;
    }
}

static int inf_stored(inf_t *s) {
    s->bitbuf = 0; s->bitcnt = 0;  /* to the byte boundary */
    if (s->pos + 4 > s->n) return -1;
    unsigned len = s->in[s->pos] | (unsigned)s->in[s->pos + 1] << 8;
    unsigned nlen = s->in[s->pos + 2] | (unsigned)s->in[s->pos + 3] << 8;
    s->pos += 4;
    if (len != (~nlen & 0xFFFF)) return -1;
    if (s->pos + len > s->n) return -1;
    for (unsigned i = 0; i < len; i++) if (inf_put(s, s->in[s->pos + i])) return -1;
    s->pos += len;
    return 0;
}

static int inf_fixed(inf_t *s) {
    static huff_t lit;
    static int built = 0;
    if (!built) {
        short l[288];
        for (int i = 0; i < 144; i++) l[i] = 8;
        for (int i = 144; i < 256; i++) l[i] = 9;
        for (int i = 256; i < 280; i++) l[i] = 7;
        for (int i = 280; i < 288; i++) l[i] = 8;
        huff_init(&lit, l, 288);
        built = 1;
    }
    return inf_codes(s, &lit, NULL, 1);
}

static const short kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

static int inf_dynamic(inf_t *s) {
    uint32_t v;
    if (inf_bits(s, 5, &v)) return -1;
    int nlit = (int)v + 257;
    if (inf_bits(s, 5, &v)) return -1;
    int ndist = (int)v + 1;
    if (inf_bits(s, 4, &v)) return -1;
    int nclen = (int)v + 4;
    if (nlit > 286 || ndist > 30) return -1;
    short len[320];
    memset(len, 0, sizeof len);
    for (int i = 0; i < nclen; i++) { if (inf_bits(s, 3, &v)) return -1; len[kOrder[i]] = (short)v; }
    huff_t h;
    if (!huff_init(&h, len, 19)) return -1;
    short bits[320];
    for (int i = 0; i < nlit + ndist;) {
        int sym = huff_decode(s, &h);
        if (sym < 0) return -1;
        if (sym < 16) { bits[i++] = (short)sym; continue; }
        int rep, nb; short b;
        if (sym == 16) { if (i == 0) return -1; rep = 3; nb = 2; b = bits[i - 1]; }
        else if (sym == 17) { rep = 3; nb = 3; b = 0; }
        else { rep = 11; nb = 7; b = 0; }
        if (inf_bits(s, nb, &v)) return -1;
        rep += (int)v;
        if (i + rep > nlit + ndist) return -1;
        while (rep--) bits[i++] = b;
    }
    huff_t lit, dist;
    if (!huff_init(&lit, bits, nlit) || !huff_init(&dist, bits + nlit, ndist)) return -1;
    return inf_codes(s, &lit, &dist, 0);
}

/* one DEFLATE stream from s->pos; the position afterwards is the byte after
 * the last bit used */
static int inflate_stream(inf_t *s) {
    s->bitbuf = 0; s->bitcnt = 0;
    for (;;) {
        uint32_t fin, type;
        if (inf_bits(s, 1, &fin) || inf_bits(s, 2, &type)) return -1;
        int e = type == 0 ? inf_stored(s) : type == 1 ? inf_fixed(s) : type == 2 ? inf_dynamic(s) : -1;
        if (e) return -1;
        if (fin) break;
    }
    s->bitbuf = 0; s->bitcnt = 0;
    return 0;
}

static uint32_t crc_tab[256];
static uint32_t crc_upd(uint32_t c, const uint8_t *p, size_t n) {
    if (!crc_tab[1])
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t x = i;
            for (int k = 0; k < 8; k++) x = (x & 1) ? 0xEDB88320u ^ (x >> 1) : x >> 1;
            crc_tab[i] = x;
        }
    c = ~c;
    for (size_t i = 0; i < n; i++) c = crc_tab[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return ~c;
}

/* gzip.NewReader + ioutil.ReadAll: 0 ok, -1 error */
int ref_gunzip(const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *outlen) {
    inf_t s = {in, n, 0, 0, 0, out, cap, 0, 0};
    for (int member = 0;; member++) {
        /* readHeader */
        if (s.pos == n) { if (member == 0) return -1; break; }  /* io.EOF: end of the members */
        if (n - s.pos < 10) return -1;
        const uint8_t *h = in + s.pos;
        if (h[0] != 0x1f || h[1] != 0x8b || h[2] != 8) return -1;
        uint8_t flg = h[3];
        uint32_t digest = crc_upd(0, h, 10);
        s.pos += 10;
        if (flg & 0x04) {
            if (n - s.pos < 2) return -1;
            size_t xl = in[s.pos] | (size_t)in[s.pos + 1] << 8;
            digest = crc_upd(digest, in + s.pos, 2);
            s.pos += 2;
            if (n - s.pos < xl) return -1;
            digest = crc_upd(digest, in + s.pos, xl);
            s.pos += xl;
        }
        for (int f = 0x08; f <= 0x10; f <<= 1) {  /* FNAME, FCOMMENT: readString */
            if (!(flg & f)) continue;
            size_t i = 0;
            for (;; i++) {
                if (i >= 512) return -1;
                if (s.pos + i >= n) return -1;
                if (in[s.pos + i] == 0) break;
            }
            digest = crc_upd(digest, in + s.pos, i + 1);
            s.pos += i + 1;
        }
        if (flg & 0x02) {
            if (n - s.pos < 2) return -1;
            unsigned hc = in[s.pos] | (unsigned)in[s.pos + 1] << 8;
            if (hc != (digest & 0xFFFF)) return -1;
            s.pos += 2;
        }
        size_t start = s.cnt;
        s.base = start;
        if (inflate_stream(&s)) return -1;
        if (n - s.pos < 8) return -1;
        const uint8_t *t = in + s.pos;
        uint32_t crc = t[0] | (uint32_t)t[1] << 8 | (uint32_t)t[2] << 16 | (uint32_t)t[3] << 24;
        uint32_t isz = t[4] | (uint32_t)t[5] << 8 | (uint32_t)t[6] << 16 | (uint32_t)t[7] << 24;
        s.pos += 8;
        if (crc != crc_upd(0, out + start, s.cnt - start) || isz != (uint32_t)(s.cnt - start)) return -1;
    }
    *outlen = s.cnt;
    return 0;
}

/* ------------------------------------------------------------ snappy */
/* snappy.Decode(nil, src) into out[0..cap); 0 ok, -1 error */
static int snappy_block(const uint8_t *src, size_t n, uint8_t *out, size_t cap, size_t *outlen) {
    /* decodedLen: binary.Uvarint */
    uint64_t v = 0;
    size_t hl = 0;
    for (int sh = 0;; sh += 7) {
        if (hl >= n) return -1;          /* buffer too small */
        uint8_t b = src[hl++];
        if (hl == 10 && b > 1) return -1; /* overflow */
        v |= (uint64_t)(b & 0x7F) << sh;
        if (b < 0x80) break;
        if (hl == 10) return -1;
    }
    if (v > 0xFFFFFFFFull) return -1;
    if (v > cap) return -1;  /* more than readMessageSet accepts */
    size_t dlen = (size_t)v, d = 0, s = hl;
    while (s < n) {
        size_t length, offset = 0;
        uint8_t tag = src[s];
        switch (tag & 3) {
        case 0: {
            uint32_t x = tag >> 2;
            if (x < 60) s++;
            else {
                size_t k = x - 59;  /* 1..4 length bytes */
                s += 1 + k;
                if (s > n) return -1;
                x = 0;
                for (size_t i = 0; i < k; i++) x |= (uint32_t)src[s - k + i] << (8 * i);
            }
            length = (size_t)x + 1;
            if (length > dlen - d || length > n - s) return -1;
            memcpy(out + d, src + s, length);
            d += length; s += length;
            continue;
        }
        case 1:
            s += 2;
            if (s > n) return -1;
            length = 4 + ((src[s - 2] >> 2) & 7);
            offset = (size_t)(src[s - 2] & 0xE0) << 3 | src[s - 1];
            break;
        case 2:
            s += 3;
            if (s > n) return -1;
            length = 1 + (src[s - 3] >> 2);
            offset = src[s - 2] | (size_t)src[s - 1] << 8;
            break;
        default:
            s += 5;
            if (s > n) return -1;
            length = 1 + (src[s - 5] >> 2);
            offset = src[s - 4] | (size_t)src[s - 3] << 8 | (size_t)src[s - 2] << 16 | (size_t)src[s - 1] << 24;
            break;
        }
        if (offset == 0 || d < offset || length > dlen - d) return -1;
        for (size_t e = d + length; d != e; d++) out[d] = out[d - offset];
    }
    if (d != dlen) return -1;
    *outlen = dlen;
    return 0;
}

/* snappyDecode (proto/snappy.go): plain snappy, or the xerial framing */
int ref_unsnappy(const uint8_t *b, size_t n, uint8_t *out, size_t cap, size_t *outlen) {
    static const uint8_t magic[8] = {0x82, 'S', 'N', 'A', 'P', 'P', 'Y', 0};
    if (n < 8 || memcmp(b, magic, 8) != 0) return snappy_block(b, n, out, cap, outlen);
    if (n < 12) return -1;  /* b[8:12] out of range: a panic in the reference */
    uint32_t ver = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11];
    if (ver != 1) return -1;
    size_t total = 0;
    for (size_t i = 16; i < n;) {
        if (n - i < 4) return -1;  /* panic in the reference */
        size_t cn = (size_t)b[i] << 24 | (size_t)b[i + 1] << 16 | (size_t)b[i + 2] << 8 | b[i + 3];
        i += 4;
        if (cn > n - i) return -1;  /* panic in the reference */
        size_t got;
        if (snappy_block(b + i, cn, out + total, cap - total, &got)) return -1;
        total += got;
        i += cn;
    }
    *outlen = total;
    return 0;
}
