// memcached request classification on gfx950 (product code).
//
// One lane per request.  The first byte picks the framing, as the parser
// selection of proxylib/memcached/parser.go:186-202 does:
//   binary (>= 0x80): the 24-byte header (binary/parser.go:58-139) gives the
//     opcode, key and frame length = body + 24;
//   text: the first "\r\n" ends the command line (text/parser.go:84-93); the
//     line is split like bytes.Fields (Unicode White_Space) and classified by
//     its first token (:101-156); storage commands add tokens[4] + 2 bytes.
// Each lane walks its line once, byte by byte, from 16-byte aligned vector
// loads held in registers.  Key tokens are fed to the rule set's key DFAs as
// they stream past, so no token offsets are stored; at the end of each key
// the DFA masks fold into an AND over keys (memcache.Rule.Matches, "every
// key", proxylib/memcached/parser.go:67-97).  The verdict is the first rule
// (in evaluation order) with  empty || (command && all keys), else the rule
// set's terminal verdict.
//
// Batch conventions (include/l7gpu.h): PASS/DROP => ALLOW/DENY
// with consumed = proxylib's frame length (it may exceed the buffer); MORE n
// => INCOMPLETE, consumed n (NOP => 0); panic / ERROR 0 => PARSE_ERROR,
// consumed 0; binary ERROR_INVALID_FRAME_TYPE => PARSE_ERROR, consumed 2; a
// frame length outside 1..2^32-1 => PARSE_ERROR.  The connection flags hold
// the parser its first byte chose (0: this buffer's first byte decides).
#include <hip/hip_runtime.h>

#include "../device_tables.h"
#include "../engine/mc_groups.h"
#include "../regex/nfa_walk.h"
#include "copy_in.h"
#include "gmem.h"
#include "service.h"

namespace l7 {

namespace {

constexpr int kBlock = 256;
// key DFAs walked per pass over the line (more DFAs: more passes)
constexpr int kMcPassDfas = 1;
constexpr uint32_t kMcLdsImages = 32 * 1024;  // LDS budget for the staged rule-set images
constexpr int kMcWaves = kBlock / 64;
constexpr int kMcSortPer = 4;                          // list entries per lane per chunk (1: 4.33 ms, 2: 3.82, 4: 3.25, 8: 3.26, 16: 4.41 on cfg5)
constexpr uint32_t kMcWaveChunk = 64 * kMcSortPer;     // entries a wave orders by parser at a time
// waves per SIMD the common kernel is built for (below)
// (round 5, with the entry fields in LDS: 4 / 5 / 6 waves -> cfg5 memcached 3.55 /
// 3.27 / 3.24 ms, the mixed 4M stream 0.242 / 0.257 / 0.275 ms; profiles/r5/ab5i_*)
constexpr int kMcWavesPerSimd = 5;

// 16-byte aligned register window over one request (the arena is readable up
// to the 16-byte boundary after its last byte; see include/l7gpu.h).
struct Reader {
    const uint8_t *b;
    uint64_t base;
    uint32_t w0, w1, w2, w3;
};

__device__ __forceinline__ uint32_t rd(Reader &r, uint32_t i) {
    const uint64_t a = (uint64_t)(r.b + i);
    const uint64_t base = a & ~(uint64_t)15;
    if (base != r.base) {
        const uint4 v = gload16(base);  // global, not flat (gmem.h)
        r.w0 = v.x; r.w1 = v.y; r.w2 = v.z; r.w3 = v.w;
        r.base = base;
    }
    const uint32_t k = (uint32_t)(a >> 2) & 3;
    const uint32_t w = k == 0 ? r.w0 : k == 1 ? r.w1 : k == 2 ? r.w2 : r.w3;
    return (w >> ((a & 3) * 8)) & 0xFF;
}

// text command name bytes packed little-endian into 4 words (compile-time)
__host__ __device__ constexpr uint32_t pk(const char *s, uint32_t n, uint32_t w) {
    return (4 * w + 0 < n ? (uint32_t)(uint8_t)s[4 * w + 0] : 0u) |
           (4 * w + 1 < n ? (uint32_t)(uint8_t)s[4 * w + 1] << 8 : 0u) |
           (4 * w + 2 < n ? (uint32_t)(uint8_t)s[4 * w + 2] << 16 : 0u) |
           (4 * w + 3 < n ? (uint32_t)(uint8_t)s[4 * w + 3] << 24 : 0u);
}
#define MC_CMD(id, lit)                                                                                   \
    if (clen == sizeof(lit) - 1 && cw[0] == pk(lit, sizeof(lit) - 1, 0) && cw[1] == pk(lit, sizeof(lit) - 1, 1) && \
        cw[2] == pk(lit, sizeof(lit) - 1, 2) && cw[3] == pk(lit, sizeof(lit) - 1, 3))                    \
        return id;

// McText id of a command token (engine/mc_groups.h); kMcOther if none.
__device__ __forceinline__ uint32_t text_id(const uint32_t cw[4], uint32_t clen) {
    MC_CMD(kMcGet, "get") MC_CMD(kMcGets, "gets") MC_CMD(kMcGat, "gat") MC_CMD(kMcGats, "gats")
    MC_CMD(kMcSet, "set") MC_CMD(kMcAdd, "add") MC_CMD(kMcReplace, "replace") MC_CMD(kMcAppend, "append")
    MC_CMD(kMcPrepend, "prepend") MC_CMD(kMcCas, "cas") MC_CMD(kMcDelete, "delete") MC_CMD(kMcIncr, "incr")
    MC_CMD(kMcDecr, "decr") MC_CMD(kMcTouch, "touch") MC_CMD(kMcSlabs, "slabs") MC_CMD(kMcLru, "lru")
    MC_CMD(kMcLruCrawler, "lru_crawler") MC_CMD(kMcStats, "stats") MC_CMD(kMcVersion, "version")
    MC_CMD(kMcMisbehave, "misbehave") MC_CMD(kMcFlushAll, "flush_all") MC_CMD(kMcCacheMemlimit, "cache_memlimit")
    MC_CMD(kMcQuit, "quit") MC_CMD(kMcWatch, "watch")
    return kMcOther;
}
#undef MC_CMD

enum : int { F_NONE = 0, F_GET, F_GAT, F_STORAGE, F_KEY1, F_NOKEY, F_BAD };

struct Image {
    const uint8_t *p;
    uint32_t nch, ndfa, terminal;
    uint32_t d0, dn;  // DFAs [d0, d0+dn) are walked in the current pass over the request
    uint32_t nnfa;    // keyRegex matchers on the NFA fallback (evaluated in the first pass)
    const uint8_t *nfa_pool;
    uint64_t *nfa_scratch;  // this lane's large-NFA state sets (null: no large NFA in the pool)
};

__device__ __forceinline__ const uint64_t *u64at(const Image &I, uint32_t off) { return (const uint64_t *)(I.p + off); }
__device__ __forceinline__ uint32_t hdr32(const Image &I, int byte_off) { return *(const uint32_t *)(I.p + byte_off); }

#define MC_OFF(field) ((int)offsetof(McImgHeader, field))

template <int kCh>
struct Keys {
    uint32_t st[kMcPassDfas];   // DFA states of the key being read
    uint64_t all[kCh];          // AND over finished keys of their pass masks
};

template <int kCh>
__device__ __forceinline__ void keys_reset(const Image &I, Keys<kCh> &K) {
#pragma unroll
    for (int d = 0; d < kMcPassDfas; d++)
        if ((uint32_t)d < I.dn) {
            const DevDfa *dd = (const DevDfa *)(I.p + kMcDfaOff) + I.d0 + d;
            K.st[d] = dd->start;
        }
}

template <int kCh>
__device__ __forceinline__ void keys_step(const Image &I, Keys<kCh> &K, uint32_t c) {
#pragma unroll
    for (int d = 0; d < kMcPassDfas; d++)
        if ((uint32_t)d < I.dn && K.st[d] != 0) {
            const DevDfa *dd = (const DevDfa *)(I.p + kMcDfaOff) + I.d0 + d;
            const uint32_t cls = I.p[dd->cls_off + c];
            K.st[d] = ((const uint16_t *)(I.p + dd->trans_off))[K.st[d] * dd->ncls + cls];
        }
}

// A key ended: AND its pass mask into K.all.  In this pass a rule passes if
// its predicate is not evaluated by the pass's DFAs (no predicate, or another
// pass owns it) or one of the pass's DFAs accepts the key.  The first pass
// also runs the NFA-fallback matchers over the key bytes b[k0, k1): a rule
// whose predicate one of them is fails if it rejects the key.
template <int kCh>
__device__ __forceinline__ void keys_nfa(const Image &I, Keys<kCh> &K, const uint8_t *b, uint32_t k0, uint32_t k1) {
    const DevNfaRef *refs = (const DevNfaRef *)(I.p + hdr32(I, MC_OFF(nfa_off)));
    for (uint32_t k = 0; k < I.nnfa; k++) {
        const DevNfaRef ref = refs[k];
        if (nfa_run(I.nfa_pool, ref.nfa, b + k0, k1 - k0, I.nfa_scratch)) continue;
        const uint64_t *own = u64at(I, ref.mask_off);
#pragma unroll
        for (int c = 0; c < kCh; c++)
            if ((uint32_t)c < I.nch) K.all[c] &= ~own[c];
    }
}

template <bool kNfa, int kCh>
__device__ __forceinline__ void keys_end(const Image &I, Keys<kCh> &K, const uint8_t *b, uint32_t k0, uint32_t k1) {
    if (kNfa && I.nnfa && I.d0 == 0) keys_nfa(I, K, b, k0, k1);
    const uint64_t *owned = u64at(I, hdr32(I, MC_OFF(owned_off)));
#pragma unroll
    for (int c = 0; c < kCh; c++) {
        if ((uint32_t)c >= I.nch) break;
        uint64_t own = 0, acc = 0;
#pragma unroll
        for (int d = 0; d < kMcPassDfas; d++)
            if ((uint32_t)d < I.dn) {
                const DevDfa *dd = (const DevDfa *)(I.p + kMcDfaOff) + I.d0 + d;
                own |= owned[(I.d0 + d) * I.nch + c];
                acc |= ((const uint64_t *)(I.p + dd->mask_off))[K.st[d] * I.nch + c];
            }
        K.all[c] &= ~own | acc;
    }
    keys_reset(I, K);
}

// First-token classification (text/parser.go:101-156)
__device__ __forceinline__ void classify_cmd(const uint32_t cw[4], uint32_t clen, int &fr, uint32_t &id) {
    id = text_id(cw, clen);
    const uint32_t p3 = cw[0] & 0xFFFFFF;
    if (clen >= 3 && p3 == ('g' | 'e' << 8 | 't' << 16)) fr = F_GET;
    else if (clen >= 3 && p3 == ('g' | 'a' << 8 | 't' << 16)) fr = F_GAT;
    else if (id >= kMcSet && id <= kMcCas) fr = F_STORAGE;
    else if (id >= kMcDelete && id <= kMcTouch) fr = F_KEY1;
    else if (id >= kMcSlabs && id <= kMcWatch) fr = F_NOKEY;
    else fr = F_BAD;
}

// ---- SWAR text tokenizer (the common case of the text path)
// bit i (0..15) set iff byte i of the chunk equals b
__device__ __forceinline__ uint32_t eq_mask(uint4 w, uint32_t b) {
    const uint32_t bb = b * 0x01010101u;
    auto e = [bb](uint32_t x) {
        const uint32_t t = x ^ bb;
        return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
    };
    auto nib = [](uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); };
    return nib(e(w.x)) | nib(e(w.y)) << 4 | nib(e(w.z)) << 8 | nib(e(w.w)) << 12;
}
// bit i set iff byte i is an ASCII white space (0x09..0x0D or 0x20: unicode.IsSpace below 0x80)
__device__ __forceinline__ uint32_t ascii_space_mask(uint4 w) {
    auto sp = [](uint32_t x) {
        const uint32_t t = x & 0x7F7F7F7Fu;
        // 0x09..0x0D: t - 0x09 < 5 per byte (no borrow across bytes: t >= 0 and the high bit is clear)
        const uint32_t ge9 = (t + 0x77777777u) & 0x80808080u;   // t >= 0x09
        const uint32_t ge14 = (t + 0x72727272u) & 0x80808080u;  // t >= 0x0E
        const uint32_t tt = t ^ 0x20202020u;
        const uint32_t is20 = ~(((tt & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | tt) & 0x80808080u;
        return ((ge9 & ~ge14) | is20) & ~x & 0x80808080u;  // high bit of the byte clear
    };
    auto nib = [](uint32_t s) { return __builtin_amdgcn_ubfe((s >> 7) * 0x204081u, 21, 4); };
    return nib(sp(w.x)) | nib(sp(w.y)) << 4 | nib(sp(w.z)) << 8 | nib(sp(w.w)) << 12;
}
__device__ __forceinline__ uint32_t chunk_byte(uint4 w, uint32_t q) {
    const bool upper = (q & 8) != 0;
    const uint32_t lo = upper ? w.z : w.x, hi = upper ? w.w : w.y;
    return __builtin_amdgcn_perm(hi, lo, (q & 7) | 0x0C0C0C00u);
}

// Text command line state
struct TextLine {
    uint32_t lf;           // position of the line's "\r\n" (found)
    bool found;
    uint32_t nt;           // tokens started
    uint32_t cw[4], clen;  // first token, packed (<= 16 bytes kept)
    int fr;
    uint32_t cmd_id;
    bool a_ok, a_bad, a_neg;  // strconv.Atoi(tokens[4])
    uint32_t a_n;
    uint64_t a_v;
};

// next byte of the first token (the first 16 are kept; selects, not an
// indexed store, so cw stays in registers)
__device__ __forceinline__ void cmd_byte(TextLine &T, uint32_t c) {
    const uint32_t v = T.clen < 16 ? c << ((T.clen & 3) * 8) : 0u, wi = T.clen >> 2;
    T.cw[0] |= wi == 0 ? v : 0u;
    T.cw[1] |= wi == 1 ? v : 0u;
    T.cw[2] |= wi == 2 ? v : 0u;
    T.cw[3] |= wi == 3 ? v : 0u;
    T.clen++;
}

__device__ __forceinline__ void atoi_step(TextLine &T, uint32_t c) {
    if (T.a_n == 0 && (c == '+' || c == '-')) { T.a_neg = c == '-'; T.a_ok = false; /* until a digit */ }
    else if (c < '0' || c > '9') { T.a_ok = false; T.a_bad = true; }
    else {
        const uint64_t d = c - '0';
        if (T.a_v > (~0ull - d) / 10) T.a_bad = true;
        else T.a_v = T.a_v * 10 + d;
        if (T.a_v > 0x7FFFFFFFFFFFFFFFull + (T.a_neg ? 1u : 0u)) T.a_bad = true;
        T.a_ok = !T.a_bad;
    }
    T.a_n++;
}

__device__ __forceinline__ bool is_key_tok(const TextLine &T) {
    return (T.fr == F_GET && T.nt >= 2) || (T.fr == F_GAT && T.nt >= 3) || ((T.fr == F_STORAGE || T.fr == F_KEY1) && T.nt == 2);
}

// The command line 16 bytes at a time: per chunk the masks of ASCII spaces,
// CR and LF give the line end (the first "\r\n") and the token runs; only the
// bytes of the tokens that matter are visited one by one (the command, the
// keys through the key DFAs, tokens[4] of a storage command), every other
// byte is passed over by mask.  The split is exactly bytes.Fields' (Unicode
// White_Space, multi-byte runes included).
template <bool kNfa, int kCh>
__device__ __forceinline__ void text_fast(const Image &I, Keys<kCh> &K, const uint8_t *b, uint32_t len, TextLine &T) {
    const uint64_t a = (uint64_t)b;
    const uint32_t a0 = (uint32_t)(a & 15);
    const uint64_t base = a - a0;
    const uint32_t end = a0 + len;  // request bytes are chunk positions [a0, end)
    bool in_tok = false, key_tok = false, prev_cr = false;
    uint32_t kstart = 0, carry = 0;  // carry: bytes of this chunk that end a space rune begun in the last one
    // the next chunk's load is in flight while this one is scanned (a request
    // read in place over PCIe -- a one-request call -- pays each load's latency)
    uint4 wn = gload16(base);  // global, not flat (gmem.h)
    for (uint32_t cb = 0; cb < end; cb += 16) {
        const uint4 w = wn;
        if (cb + 16 < end) wn = gload16(base + cb + 16);
        uint32_t valid = end >= cb + 16 ? 0xFFFFu : (1u << (end - cb)) - 1u;
        if (cb == 0) valid &= 0xFFFFu << a0;
        uint32_t S = ascii_space_mask(w) | carry;
        const uint32_t CR = eq_mask(w, '\r'), LF = eq_mask(w, '\n');
        carry = 0;
        // multi-byte White_Space runes (unicode.IsSpace): U+0085, U+00A0 (C2 xx),
        // U+1680 (E1 9A 80), U+2000-U+200A, U+2028, U+2029, U+202F (E2 80 xx),
        // U+205F (E2 81 9F), U+3000 (E3 80 80).  Their lead bytes never continue
        // another rune, so each is judged on its own, as bytes.Fields' decoder
        // meets it (the bytes are in this chunk or the next)
        uint32_t lead = (eq_mask(w, 0xC2) | eq_mask(w, 0xE1) | eq_mask(w, 0xE2) | eq_mask(w, 0xE3)) & valid;
        if (lead) {
            uint4 wn = make_uint4(0, 0, 0, 0);
            if (lead >> 14 && cb + 16 < end) wn = gload16(base + cb + 16);  // holds a request byte: same page
            while (lead) {
                const uint32_t i = (uint32_t)__builtin_ctz(lead);
                lead &= lead - 1;
                const uint32_t r = cb + i - a0;  // request position
                const uint32_t c0 = chunk_byte(w, i);
                const uint32_t c1 = i + 1 < 16 ? chunk_byte(w, i + 1) : chunk_byte(wn, i - 15);
                const uint32_t c2 = i + 2 < 16 ? chunk_byte(w, i + 2) : chunk_byte(wn, i - 14);
                uint32_t L = 0;
                if (c0 == 0xC2) {
                    if (r + 1 < len && (c1 == 0x85 || c1 == 0xA0)) L = 2;
                } else if (r + 2 < len) {
                    if ((c0 == 0xE1 && c1 == 0x9A && c2 == 0x80) || (c0 == 0xE3 && c1 == 0x80 && c2 == 0x80) ||
                        (c0 == 0xE2 && ((c1 == 0x80 && ((c2 >= 0x80 && c2 <= 0x8A) || c2 == 0xA8 || c2 == 0xA9 || c2 == 0xAF)) ||
                                        (c1 == 0x81 && c2 == 0x9F))))
                        L = 3;
                }
                const uint32_t bits = ((1u << L) - 1u) << i;
                S |= bits & 0xFFFFu;
                carry |= bits >> 16;
            }
        }
        // the line end: a CR whose next byte is LF (the CR possibly the previous chunk's last byte)
        uint32_t le = 16;  // first byte of "\r\n" in this chunk (16: none; -1 handled by prev_cr)
        bool ended = false;
        if (prev_cr && (LF & valid & 1u)) {
            T.found = true;
            T.lf = cb - 1 - a0;
            ended = true;
            le = 0;  // nothing of this chunk is on the line
        } else {
            const uint32_t crlf = CR & (LF >> 1) & valid & (valid >> 1);
            if (crlf) {
                le = (uint32_t)__builtin_ctz(crlf);
                T.found = true;
                T.lf = cb + le - a0;
                ended = true;
            }
        }
        const uint32_t line = valid & ((1u << le) - 1u);  // this chunk's bytes on the line
        uint32_t m = ~S & line;  // token bytes
        uint32_t q = 0;          // next position of this chunk to look at
        for (;;) {
            if (!in_tok) {
                const uint32_t mm = m & (0xFFFFu << q);
                if (!mm) break;
                q = (uint32_t)__builtin_ctz(mm);
                T.nt++;
                key_tok = is_key_tok(T);
                kstart = cb + q - a0;
                in_tok = true;
            }
            // token bytes [q, e) of this chunk
            const uint32_t e = (uint32_t)__builtin_ctz((~m & (0xFFFFu << q)) | 0x10000u);
            if (T.nt == 1) {
                for (uint32_t k = q; k < e; k++) cmd_byte(T, chunk_byte(w, k));
            } else if (key_tok) {
                for (uint32_t k = q; k < e; k++) keys_step(I, K, chunk_byte(w, k));
            } else if (T.fr == F_STORAGE && T.nt == 5) {
                for (uint32_t k = q; k < e; k++) atoi_step(T, chunk_byte(w, k));
            }
            // the token closes at e: a space on the line, or the line end
            const bool closes = e < 16 && (((line >> e) & 1u) || (ended && e == le));
            if (!closes) break;  // it runs on into the next chunk (or the data ends)
            if (T.nt == 1) classify_cmd(T.cw, T.clen, T.fr, T.cmd_id);
            if (key_tok) keys_end<kNfa, kCh>(I, K, b, kstart, cb + e - a0);
            in_tok = false;
            q = e;
        }
        if (ended) return;
        prev_cr = (CR & valid) >> 15;
    }
    // the data ends before any "\r\n": incomplete (T.found false)
}

}  // namespace

// One request.  answer_other: answer entries on connections that are not
// memcached (single-protocol engines, where partition_kernel does not run).
// kNfa: the variant that also runs NFA-fallback key matchers (launched only
// when some memcache rule set has them; the other keeps its registers).
// kLds: `images` is the workgroup's LDS copy.  The two cases are separate
// instantiations so that every image read compiles to a ds_read (LDS) or a
// global_load: one pointer that may be either makes them all flat loads.
// mc_body: the request's offset, length and connection already in hand.
template <bool kNfa, bool kLds, int kCh>
__device__ __forceinline__ void mc_body(const Batch &B, const McTables &T, const uint8_t *images, uint32_t idx,
                                        uint64_t off, uint32_t len, DevConn conn, uint32_t answer_other) {
    {
        if (conn.proto != PROTO_MEMCACHE || conn.ruleset < 0 || (uint32_t)conn.ruleset >= T.nrulesets) {
            if (answer_other && (!L7_PROTO_OWNED(conn.proto) || conn.proto == PROTO_MEMCACHE)) {  // no parser: UNSUPPORTED
                B.verdict[idx] = V_UNSUPPORTED;
                B.rule[idx] = -1;
                B.consumed[idx] = 0;
            }
            return;
        }
        const DevRuleset rs = T.rulesets[conn.ruleset];
        Image I;
        I.p = images + rs.image_off;
        {
            const uint32_t h0 = *(const uint32_t *)I.p;
            I.nch = h0 & 0xFF;
            I.terminal = (h0 >> 8) & 0xFF;
            I.ndfa = (h0 >> 16) & 0xFF;
        }
        I.nnfa = hdr32(I, MC_OFF(nnfa));
        I.nfa_pool = T.nfa_pool;
        I.nfa_scratch = kNfa ? l7_nfa_lane_scratch(T.nfa_scratch, T.nfa_lane_words) : nullptr;
        const uint8_t *b = B.arena + off;
        uint8_t verdict = V_PARSE_ERROR;
        int32_t rule = -1;
        uint32_t consumed = 0;
        const bool in_arena = l7_in_arena(off, len, B.arena_len);
        Keys<kCh> K;
#pragma unroll
        for (int c = 0; c < kCh; c++) K.all[c] = ~0ull;
        const uint64_t *cmdmask = nullptr;
        uint64_t frame = 0;
        bool staged = false;  // framing succeeded: match against the rules
        // More key DFAs than one pass walks: re-read the request once per
        // group of kMcPassDfas (framing is identical in every pass).
        if (!in_arena) verdict = V_UNSUPPORTED;  // out of contract: nothing is read
        for (uint32_t d0 = 0; in_arena; d0 += kMcPassDfas) {
        I.d0 = d0;
        I.dn = I.ndfa - d0 < (uint32_t)kMcPassDfas ? I.ndfa - d0 : (uint32_t)kMcPassDfas;
        keys_reset(I, K);
        do {
            uint32_t mode = conn.flags & 3;
            if (len == 0 && mode == 0) { verdict = V_INCOMPLETE; break; }  // NOP, 0
            if (mode == 0) mode = b[0] >= 0x80 ? 2 : 1;
            if (mode == 2) {
                // ---- binary header (binary/parser.go:72-139)
                if (len < 24) { verdict = V_INCOMPLETE; consumed = 24 - len; break; }  // MORE headerMissing
                const uint32_t keylen = (uint32_t)b[2] << 8 | b[3];
                const uint32_t extras = b[4];
                const uint32_t body = (uint32_t)b[8] << 24 | (uint32_t)b[9] << 16 | (uint32_t)b[10] << 8 | b[11];
                if (keylen > 0 && 24 + keylen + extras > len) {  // MORE keyMissing
                    verdict = V_INCOMPLETE;
                    consumed = 24 + keylen + extras - len;
                    break;
                }
                if ((b[0] & 0x80) == 0) { consumed = 2; break; }  // ERROR, ERROR_INVALID_FRAME_TYPE
                cmdmask = u64at(I, hdr32(I, MC_OFF(op_off))) + (size_t)b[1] * I.nch;
                Reader R{b, ~0ull, 0, 0, 0, 0};
                for (uint32_t i = 24 + extras, e = 24 + extras + keylen; i < e; i++) keys_step(I, K, rd(R, i));
                keys_end<kNfa, kCh>(I, K, b, 24 + extras, 24 + extras + keylen);
                frame = (uint32_t)(body + 24u);  // uint32 arithmetic, then int()
            } else {
                // ---- text command line
                TextLine T;
                T.lf = 0;
                T.found = false;
                T.nt = 0;
                T.cw[0] = T.cw[1] = T.cw[2] = T.cw[3] = 0;
                T.clen = 0;
                T.fr = F_NONE;
                T.cmd_id = kMcOther;
                T.a_ok = T.a_bad = T.a_neg = false;
                T.a_n = 0;
                T.a_v = 0;
                text_fast<kNfa, kCh>(I, K, b, len, T);
                if (!T.found) {  // MORE 1 if the data ends in '\r', else MORE 2
                    verdict = V_INCOMPLETE;
                    consumed = (len > 0 && b[len - 1] == '\r') ? 1 : 2;
                    break;
                }
                const uint32_t nt = T.nt;
                const int fr = T.fr;
                if (nt == 0) break;  // tokens[0] panics
                if (fr == F_BAD) break;  // ERROR, 0
                if (fr == F_GAT && nt < 2) break;  // tokens[2:] panics
                if ((fr == F_STORAGE || fr == F_KEY1) && nt < 2) break;  // tokens[1:2] panics
                frame = (uint64_t)T.lf + 2;
                if (fr == F_STORAGE) {
                    if (nt < 5) break;  // tokens[4] panics
                    if (!T.a_ok) break;
                    const int64_t nb = T.a_neg ? (int64_t)(0 - T.a_v) : (int64_t)T.a_v;
                    frame = frame + (uint64_t)nb + 2u;  // Go int arithmetic
                }
                cmdmask = u64at(I, hdr32(I, MC_OFF(text_off))) + (size_t)T.cmd_id * I.nch;
            }
            staged = true;
        } while (false);
        if (!staged || d0 + kMcPassDfas >= I.ndfa) break;
        }
        do {
            if (!staged) break;
            if ((int64_t)frame <= 0 || frame > 0xFFFFFFFFull) { verdict = V_PARSE_ERROR; break; }
            consumed = (uint32_t)frame;
            // ---- first matching rule (PortNetworkPolicyRule(s).Matches order)
            const uint64_t *empty = u64at(I, hdr32(I, MC_OFF(empty_off)));
            const int32_t *ids = (const int32_t *)(I.p + hdr32(I, MC_OFF(rule_off)));
            verdict = (uint8_t)I.terminal;
#pragma unroll
            for (int c = 0; c < kCh; c++) {
                if ((uint32_t)c >= I.nch) break;
                const uint64_t ok = empty[c] | (cmdmask[c] & K.all[c]);
                if (ok) { verdict = V_ALLOW; rule = ids[c * 64 + __builtin_ctzll(ok)]; break; }
            }
        } while (false);
        B.verdict[idx] = verdict;
        B.rule[idx] = rule;
        B.consumed[idx] = consumed;
    }
}

template <bool kNfa, bool kLds, int kCh>
__device__ __forceinline__ void mc_one(const Batch &B, const McTables &T, const uint8_t *images, uint32_t idx,
                                       uint32_t answer_other) {
    // the request's connection, offset and length in one round trip (for a
    // one-request call they come over PCIe), then its connection
    const uint32_t ci = B.conn_ids[idx];
    const uint64_t off = B.offs[idx];
    const uint32_t len = B.lens[idx];
    const DevConn conn = ci < B.nconns ? B.conns[ci] : DevConn{-1, PROTO_NONE, 0, 0xFFFF};
    mc_body<kNfa, kLds, kCh>(B, T, images, idx, off, len, conn, answer_other);
}

// The parser each of a lane's kMcSortPer entries takes (memcached/parser.go:
// 186-202: the connection's, else the one its first byte picks), and text
// retrievals (get / gets / gat / gats) apart from the other commands, whose
// lines are longer and parse more tokens: 0 text retrieval, 1 other text, 2
// binary, 3 everything else, 4 no entry.  The loads go out phase by phase
// (connection ids, connections, offsets / lengths, first bytes) so the lane
// waits four memory latencies, not four per entry.
// Also returned, for the classifying lane (no second fetch): the entry's
// offset, length and connection (rsf: rule set << 12 | flags << 10 | offset
// bits 32..41; ~0u: kind 3, or a field that does not fit, and the
// classifying lane reads them itself).
__device__ __forceinline__ void mc_kinds(const Batch &B, const McTables &T, const uint32_t (&ix)[kMcSortPer],
                                         uint32_t (&kd)[kMcSortPer], uint64_t (&of)[kMcSortPer],
                                         uint32_t (&ln)[kMcSortPer], uint32_t (&rsf)[kMcSortPer]) {
    uint32_t ci[kMcSortPer], fl[kMcSortPer];
#pragma unroll
    for (int r = 0; r < kMcSortPer; r++) ci[r] = ix[r] != ~0u ? B.conn_ids[ix[r]] : ~0u;
#pragma unroll
    for (int r = 0; r < kMcSortPer; r++) {
        kd[r] = ix[r] == ~0u ? 4 : 3;
        fl[r] = 0;
        rsf[r] = ~0u;
        if (ci[r] < B.nconns) {
            const DevConn c = B.conns[ci[r]];
            if (c.proto == PROTO_MEMCACHE && c.ruleset >= 0 && (uint32_t)c.ruleset < T.nrulesets) {
                kd[r] = 0;
                fl[r] = c.flags;
                rsf[r] = c.ruleset < (1 << 20) ? (uint32_t)c.ruleset << 12 | (c.flags & 3u) << 10 : ~0u;
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kMcSortPer; r++) {
        of[r] = 0;
        ln[r] = 0;
        if (kd[r] == 0) {
            of[r] = B.offs[ix[r]];
            ln[r] = B.lens[ix[r]];
            if (ln[r] == 0 || !l7_in_arena(of[r], ln[r], B.arena_len)) {
                kd[r] = 3;
                rsf[r] = ~0u;
            } else if (rsf[r] != ~0u) {
                rsf[r] = of[r] >> 42 ? ~0u : rsf[r] | (uint32_t)(of[r] >> 32);  // (offsets past 4 TiB: fetched again)
            }
        }
    }
#pragma unroll
    for (int r = 0; r < kMcSortPer; r++) {
        if (kd[r] != 0) continue;
        const uint32_t b0 = B.arena[of[r]];
        uint32_t mode = fl[r] & 3;
        if (mode == 0) mode = b0 >= 0x80 ? 2 : 1;
        kd[r] = mode == 2 ? 2 : b0 == 'g' ? 0 : 1;
    }
}

// sel: this protocol's request indices (partition_kernel, mixed batches), else
// requests 0..n-1.  Each wave takes kMcWaveChunk list entries at a time,
// reads each one's parser from its first byte (a line the classification
// reads next anyway), orders them by parser in its own LDS slice (stable:
// list order within a parser), then classifies them in that order, so the
// wave mostly runs one parser's path instead of text and binary one after the
// other.  The slice holds each entry's index, length, offset and connection
// (16 bytes), so the classifying lane starts from the rule set and the
// request's bytes instead of fetching the entry's metadata a second time.
// Waves never wait for each other (no workgroup barrier).
template <bool kNfa, bool kLds, int kCh>
__device__ __forceinline__ void mc_loop(Batch B, McTables T, const uint8_t *images, const uint32_t *__restrict__ sel,
                                        const uint32_t *__restrict__ sel2, const uint32_t *__restrict__ sel_count,
                                        uint32_t answer_other, uint4 *ent) {
    const uint32_t n = B.n;
    // sel: sel_count[0] entries from sel's start, sel_count[1] from its end,
    // sel_count[3] from sel2's end (n slots each); null: all n
    const uint32_t ma = sel ? sel_count[0] : n;
    const uint32_t mb = sel ? ma + sel_count[3] : n;
    const uint32_t m = sel ? mb + sel_count[1] : n;
    const uint32_t lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (m <= 64) {  // one wave's worth (a proxylib OnData): nothing to order, and the
                    // first bytes would be one more round trip (zero-copy: over PCIe)
        const uint32_t i = lane;
        if (blockIdx.x == 0 && wave == 0 && i < m)
            mc_one<kNfa, kLds, kCh>(B, T, images, !sel ? i : i < ma ? sel[i] : i < mb ? sel2[n - 1 - (i - ma)] : sel[n - 1 - (i - mb)],
                                    answer_other);
        return;
    }
    const uint64_t below = (1ull << lane) - 1;
    uint4 *slot = ent + wave * kMcWaveChunk;
    for (uint32_t base = (blockIdx.x * kMcWaves + wave) * kMcWaveChunk; base < m;
         base += gridDim.x * kMcWaves * kMcWaveChunk) {
        uint32_t ix[kMcSortPer], kd[kMcSortPer], ln[kMcSortPer], rsf[kMcSortPer];
        uint64_t of[kMcSortPer];
#pragma unroll
        for (int r = 0; r < kMcSortPer; r++) {
            const uint32_t i = base + r * 64 + lane;
            ix[r] = i >= m ? ~0u : !sel ? i : i < ma ? sel[i] : i < mb ? sel2[n - 1 - (i - ma)] : sel[n - 1 - (i - mb)];
        }
        mc_kinds(B, T, ix, kd, of, ln, rsf);
        uint32_t lo[4] = {0, 0, 0, 0};  // exclusive offsets, parser-major
#pragma unroll
        for (int r = 0; r < kMcSortPer; r++)
#pragma unroll
            for (int k = 0; k < 3; k++) lo[k + 1] += __popcll(__ballot(kd[r] <= (uint32_t)k));
#pragma unroll
        for (int r = 0; r < kMcSortPer; r++) {
#pragma unroll
            for (int k = 0; k < 4; k++) {
                const uint64_t mk = __ballot(kd[r] == (uint32_t)k);
                if (kd[r] == (uint32_t)k) slot[lo[k] + __popcll(mk & below)] = make_uint4(ix[r], ln[r], (uint32_t)of[r], rsf[r]);
                lo[k] += __popcll(mk);
            }
        }
        const uint32_t total = min(m - base, kMcWaveChunk);
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        for (uint32_t k = lane; k < total; k += 64) {
            const uint4 e = slot[k];  // {index, length, offset low, offset high 10 bits | rule set << 12 | flags << 10}
            if (e.w == ~0u) {
                mc_one<kNfa, kLds, kCh>(B, T, images, e.x, answer_other);
            } else {
                const DevConn conn{(int32_t)(e.w >> 12), PROTO_MEMCACHE, (uint8_t)((e.w >> 10) & 3u), 0xFFFF};
                mc_body<kNfa, kLds, kCh>(B, T, images, e.x, (uint64_t)(e.w & 0x3FFu) << 32 | e.z, e.y, conn,
                                         answer_other);
            }
        }
        __builtin_amdgcn_wave_barrier();  // (the slice is rewritten by the next chunk)
    }
}

// The rule-set images (command / opcode masks, key DFAs) are read once per
// key byte in a dependent chain: when they all fit, every workgroup stages
// them in LDS and walks them there instead of through L1/L2.
__device__ __forceinline__ void mc_stage_images(const McTables &T, uint8_t *lds) {
    const uint32_t n16 = (T.images_len + 15) / 16;
    // every load issued before the first store: one memory round trip per
    // 32 KiB, not one per 4 KiB (a one-request launch waits on this)
    constexpr uint32_t kIters = 8;  // kMcLdsImages / (16 * kBlock)
    static_assert(kIters * 16 * kBlock == kMcLdsImages, "staging rounds");
    uint4 t[kIters];
#pragma unroll
    for (uint32_t k = 0; k < kIters; k++)
        if (threadIdx.x + k * kBlock < n16) t[k] = ((const uint4 *)T.images)[threadIdx.x + k * kBlock];
#pragma unroll
    for (uint32_t k = 0; k < kIters; k++)
        if (threadIdx.x + k * kBlock < n16) ((uint4 *)lds)[threadIdx.x + k * kBlock] = t[k];
    __syncthreads();
}
__device__ __forceinline__ bool mc_images_fit(const McTables &T) { return T.images_len && T.images_len <= kMcLdsImages; }

template <bool kNfa, int kCh>
__device__ __forceinline__ void mc_classify(Batch B, McTables T, const uint32_t *__restrict__ sel,
                                            const uint32_t *__restrict__ sel2, const uint32_t *__restrict__ sel_count,
                                            uint32_t answer_other, const CopyIn &ci) {
    copy_in_block(ci);  // (a one-workgroup call's inputs, when the host asks)
    extern __shared__ __attribute__((aligned(16))) uint8_t mc_lds[];
    __shared__ uint4 s_ent[kMcWaves][kMcWaveChunk];  // each wave's entries in parser order, with their fields
    if (mc_images_fit(T)) {
        mc_stage_images(T, mc_lds);
        mc_loop<kNfa, true, kCh>(B, T, mc_lds, sel, sel2, sel_count, answer_other, &s_ent[0][0]);
    } else {
        mc_loop<kNfa, false, kCh>(B, T, T.images, sel, sel2, sel_count, answer_other, &s_ent[0][0]);
    }
    signal_done_block(ci);
}

// The resident service (kernels/service.h) for the synchronous memcached calls
// (one proxylib OnData): each posted call's inputs copied into HBM, mc_loop
// over them (at most 64 requests: one wave, no parser ordering), the answers
// to pinned memory, then the done word; the images staged in LDS once for
// the service's lifetime.
template <int kCh>
__global__ __launch_bounds__(kBlock) void memcache_service_kernel(SvcBox *box, SvcStatic S, McTables T, uint32_t seen0,
                                                                  uint64_t idle) {
    __shared__ __attribute__((aligned(16))) uint8_t lds[kMcLdsImages];
    __shared__ uint4 s_ent[kMcWaves][kMcWaveChunk];
    uint32_t *word = reinterpret_cast<uint32_t *>(&s_ent[0][0]);  // (the entries' slice: unused between calls)
    uint32_t seen = seen0;
    uint64_t t_last = __builtin_amdgcn_s_memtime();
    const bool fit = mc_images_fit(T);
    if (fit) mc_stage_images(T, lds);
    if (threadIdx.x == 0) svc_store(&box->state, kSvcRunning);
    for (;;) {
        const SvcCall c = svc_next(box, seen, t_last, idle, word);
        if (!c.seq) break;
        const Batch B = svc_batch(S, c);
        const CopyIn ci = svc_copy(S, box, c);
        copy_in_block(ci);
        const uint32_t other = (c.flags & kSvcAnswerOther) ? 1u : 0u;
        if (fit) mc_loop<false, true, kCh>(B, T, lds, nullptr, nullptr, nullptr, other, &s_ent[0][0]);
        else mc_loop<false, false, kCh>(B, T, T.images, nullptr, nullptr, nullptr, other, &s_ent[0][0]);
        signal_done_block(ci);
        __syncthreads();
        t_last = __builtin_amdgcn_s_memtime();
    }
    if (threadIdx.x == 0) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "");
        svc_store(&box->state, kSvcStopped);
    }
}

// The common kernel is built for kMcWavesPerSimd waves per SIMD (round 3 on 2.4M
// mixed-stream memcached requests: 4 waves (100 VGPRs, no spill) 0.91 ms,
// 6 waves 0.79-0.82, 7 waves 0.79, 8 waves 0.84 -- the spills grow);
// the NFA variant keeps its registers.
// kCh: 64-rule chunks the kernel carries per request (1 when every rule set
// has at most 64 rules: 6 fewer registers per lane than the 4-chunk build).
// (the 4-chunk build holds 6 more registers: 4 waves per SIMD, where it does not spill)
template <int kCh>
__global__ __launch_bounds__(kBlock) __attribute__((amdgpu_waves_per_eu(kCh == 1 ? kMcWavesPerSimd : 4, 8))) void memcache_classify_kernel(Batch B, McTables T,
                                                                                  const uint32_t *__restrict__ sel,
                                                                                  const uint32_t *__restrict__ sel2,
                                                                                  const uint32_t *__restrict__ sel_count,
                                                                                  uint32_t answer_other, CopyIn ci) {
    mc_classify<false, kCh>(B, T, sel, sel2, sel_count, answer_other, ci);
}
__global__ __launch_bounds__(kBlock) void memcache_classify_nfa_kernel(Batch B, McTables T,
                                                                       const uint32_t *__restrict__ sel,
                                                                       const uint32_t *__restrict__ sel2,
                                                                       const uint32_t *__restrict__ sel_count,
                                                                       uint32_t answer_other, CopyIn ci) {
    mc_classify<true, kMcMaxChunks>(B, T, sel, sel2, sel_count, answer_other, ci);
}

// scratch_lanes: lanes T.nfa_scratch holds (when it is set)
hipError_t LaunchMemcacheClassify(const Batch &B, const McTables &T, const uint32_t *sel, const uint32_t *sel2,
                                  const uint32_t *sel_count, bool answer_other, uint32_t scratch_lanes,
                                  hipStream_t stream, const CopyIn *ci) {
    if (B.n == 0) return hipSuccess;
    // (cfg5, 20M entries: caps of 2048 / 4096 / 8192 / 16384 / 32768 / 131072
    // workgroups -> 3.62 / 3.39 / 3.26 / 3.21 / 3.25 / 3.72 ms; profiles/r5/ab5l_*)
    uint32_t blocks = (B.n + kBlock - 1) / kBlock;
    if (blocks > 16384) blocks = 16384;
    if (T.nfa_scratch) blocks = max(1u, min(blocks, scratch_lanes / kBlock));  // (grid-stride loop)
    if (ci && blocks != 1) return hipErrorInvalidValue;  // (the copy is one workgroup's)
    const CopyIn c = ci ? *ci : CopyIn{};
    const size_t lds = T.images_len && T.images_len <= kMcLdsImages ? ((T.images_len + 15) & ~15u) : 0;
    if (T.nfa_pool)
        hipLaunchKernelGGL(memcache_classify_nfa_kernel, dim3(blocks), dim3(kBlock), lds, stream, B, T, sel, sel2, sel_count,
                           answer_other ? 1u : 0u, c);
    else if (T.max_chunks <= 1)
        hipLaunchKernelGGL(memcache_classify_kernel<1>, dim3(blocks), dim3(kBlock), lds, stream, B, T, sel, sel2, sel_count,
                           answer_other ? 1u : 0u, c);
    else
        hipLaunchKernelGGL(memcache_classify_kernel<kMcMaxChunks>, dim3(blocks), dim3(kBlock), lds, stream, B, T, sel, sel2,
                           sel_count, answer_other ? 1u : 0u, c);
    return hipGetLastError();
}

// The memcached service: one workgroup on `stream` until it leaves (idle
// cycles without a call, or stop).  Calls of at most 64 requests (one wave).
hipError_t LaunchMemcacheService(SvcBox *box, const SvcStatic &S, const McTables &T, uint32_t seen0, uint64_t idle,
                                 hipStream_t stream) {
    if (T.nfa_pool) return hipErrorInvalidValue;  // (NFA key matchers: the launched path)
    if (T.max_chunks <= 1)
        hipLaunchKernelGGL(memcache_service_kernel<1>, dim3(1), dim3(kBlock), 0, stream, box, S, T, seen0, idle);
    else
        hipLaunchKernelGGL(memcache_service_kernel<kMcMaxChunks>, dim3(1), dim3(kBlock), 0, stream, box, S, T, seen0,
                           idle);
    return hipGetLastError();
}

}  // namespace l7
