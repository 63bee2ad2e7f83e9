// Bit-parallel NFA walk (product code): the one implementation of the
// DevNfa step (device_tables.h), compiled for the gfx950 pre-pass kernels and
// for the host-side test hook (l7g_debug_regex with the NFA forced), so the
// tables the device walks are checked on the CPU as they are.
//
// Semantics (re_dfa.h BitNfa): Go regexp over raw bytes with utf8.DecodeRune's
// rune boundaries and empty-width assertions; full match when the pattern was
// compiled anchored, regexp.Match otherwise.
#pragma once
#include <stdint.h>

#include "../device_tables.h"

#if defined(__HIPCC__)
#define L7_NFA_INL __host__ __device__ __forceinline__
#else
#define L7_NFA_INL inline
#endif

namespace l7 {

// empty-width condition bits (the C_* of re_dfa.cc) and previous-byte context
enum : uint32_t { NC_BOT = 1, NC_EOT = 2, NC_BOL = 4, NC_EOL = 8, NC_WB = 16, NC_NWB = 32 };
enum : uint32_t { NP_START = 1, NP_NL = 2, NP_WORD = 4 };

L7_HD inline bool nfa_word_byte(uint32_t b) {
    return (b - '0' < 10u) || ((b | 0x20) - 'a' < 26u) || b == '_';
}
// condition at the boundary before byte b (b < 0: end of text)
L7_HD inline uint32_t nfa_cond(uint32_t prev, int b) {
    uint32_t c = 0;
    if (prev & NP_START) c |= NC_BOT | NC_BOL;
    if (prev & NP_NL) c |= NC_BOL;
    const bool pw = (prev & NP_WORD) != 0;
    if (b < 0) return c | NC_EOT | NC_EOL | (pw ? NC_WB : NC_NWB);
    if (b == '\n') c |= NC_EOL;
    return c | ((pw != nfa_word_byte((uint32_t)b)) ? NC_WB : NC_NWB);
}
// utf8.DecodeRune(s[i:n]): the rune and its width (an invalid or truncated
// sequence is U+FFFD of width 1)
L7_HD inline uint32_t nfa_decode(const uint8_t *s, uint32_t i, uint32_t n, uint32_t *width) {
    const uint32_t c = s[i];
    *width = 1;
    if (c < 0x80) return c;
    if (c < 0xC2 || c > 0xF4) return 0xFFFD;
    const uint32_t need = c < 0xE0 ? 1 : c < 0xF0 ? 2 : 3;
    uint32_t lo = 0x80, hi = 0xBF;
    if (c == 0xE0) lo = 0xA0;
    else if (c == 0xED) hi = 0x9F;
    else if (c == 0xF0) lo = 0x90;
    else if (c == 0xF4) hi = 0x8F;
    if (n - i <= need) return 0xFFFD;
    const uint32_t b1 = s[i + 1];
    if (b1 < lo || b1 > hi) return 0xFFFD;
    uint32_t r = (c & (0x7Fu >> (need + 1))) << 6 | (b1 & 0x3F);
    for (uint32_t k = 2; k <= need; k++) {
        const uint32_t b = s[i + k];
        if (b - 0x80u > 0x3Fu) return 0xFFFD;
        r = r << 6 | (b & 0x3F);
    }
    *width = need + 1;
    return r;
}

// Rune interval (the ASCII table, else the last interval starting at or below r)
L7_HD inline uint32_t nfa_interval(const uint8_t *pool, const DevNfa *d, uint32_t r) {
    if (r < 128) return ((const uint16_t *)(pool + d->ascii_off))[r];
    const uint32_t *ivl = (const uint32_t *)(pool + d->ivl_off);
    uint32_t lo = 0, hi = d->nivl;
    while (hi - lo > 1) {
        const uint32_t mid = (lo + hi) >> 1;
        if (ivl[mid] <= r) lo = mid;
        else hi = mid;
    }
    return lo;
}

// ---- large NFAs (W > kNfaMaxWords: sparse rows, device_tables.h
// DevNfaSparse).  The two state sets live in the caller's scratch (2 W words
// per lane); only the words [lo, hi] of the current set are live, and the
// next set is cleared lazily over the words its rows touch.
L7_HD inline bool nfa_big_step(const uint8_t *pool, const DevNfa *d, const uint64_t *S, uint64_t *N, uint32_t &lo,
                               uint32_t &hi, uint32_t k, uint32_t iv) {
    const DevNfaSparse *sp = (const DevNfaSparse *)(pool + d->t_off);
    const uint32_t *row_of = (const uint32_t *)(pool + sp->row_of_off) + (size_t)k * d->m;
    const uint32_t *row_ptr = (const uint32_t *)(pool + sp->row_ptr_off);
    const uint32_t *pw = (const uint32_t *)(pool + sp->pair_w_off);
    const uint64_t *pm = (const uint64_t *)(pool + sp->pair_m_off);
    uint32_t nlo = 1, nhi = 0;  // (empty)
    for (uint32_t w = lo; w <= hi; w++) {
        uint64_t x = S[w];
        while (x) {
            const uint32_t p = w * 64 + (uint32_t)__builtin_ctzll(x);
            x &= x - 1;
            const uint32_t row = row_of[p];
            for (uint32_t e = row_ptr[row], ee = row_ptr[row + 1]; e < ee; e++) {
                const uint32_t u = pw[e];
                if (nlo > nhi) {
                    N[u] = 0;
                    nlo = nhi = u;
                } else if (u < nlo) {
                    for (uint32_t z = u; z < nlo; z++) N[z] = 0;
                    nlo = u;
                } else if (u > nhi) {
                    for (uint32_t z = nhi + 1; z <= u; z++) N[z] = 0;
                    nhi = u;
                }
                N[u] |= pm[e];
            }
        }
    }
    if (nlo > nhi) return false;
    const uint64_t *B = (const uint64_t *)(pool + d->b_off) + (size_t)iv * d->W;
    uint32_t a = 1, b = 0;
    for (uint32_t u = nlo; u <= nhi; u++) {
        const uint64_t v = N[u] & B[u];
        N[u] = v;
        if (v) {
            if (a > b) a = u;
            b = u;
        }
    }
    if (a > b) return false;
    lo = a;
    hi = b;
    return true;
}

L7_HD inline bool nfa_big_accepts(const uint8_t *pool, const DevNfa *d, const uint64_t *S, uint32_t lo, uint32_t hi,
                                  uint32_t k) {
    const uint64_t *Acc = (const uint64_t *)(pool + d->acc_off) + (size_t)k * d->W;
    uint64_t hit = 0;
    for (uint32_t u = lo; u <= hi; u++) hit |= S[u] & Acc[u];
    return hit != 0;
}

// Streaming walk (for text the caller produces rune by rune, e.g. the
// lowered cassandra table name): nfa_begin, one nfa_step per rune (r, and c =
// the first byte of its encoding, which the empty-width conditions look at),
// nfa_end.  Same step as nfa_run below, which keeps its own loop so its state
// stays in registers in the pre-pass kernels.
struct NfaRun {
    uint64_t S[kNfaMaxWords];
    uint32_t prev;
    bool dead;
    uint64_t *big;     // a large NFA's two state sets (2 W words of scratch; null: none given)
    uint32_t cur, lo, hi;
};

// scratch: 2 W words when the NFA may be a large one (see nfa_run)
L7_NFA_INL void nfa_begin(NfaRun &R, uint64_t *scratch = nullptr) {
#pragma unroll
    for (int w = 0; w < kNfaMaxWords; w++) R.S[w] = w == 0 ? 1 : 0;  // the virtual start position
    R.prev = NP_START;
    R.dead = false;
    R.big = scratch;
    R.cur = 0;
    R.lo = R.hi = 0;
    if (scratch) scratch[0] = 1;
}

L7_NFA_INL void nfa_step(const uint8_t *pool, uint64_t off, NfaRun &R, uint32_t r, uint32_t c) {
    if (R.dead) return;
    const DevNfa *d = (const DevNfa *)(pool + off);
    if (d->W > (uint32_t)kNfaMaxWords) {
        if (!R.big) {  // (the launcher gives scratch whenever the pool holds a large NFA)
            R.dead = true;
            return;
        }
        uint64_t *S = R.big + (size_t)R.cur * d->W, *N = R.big + (size_t)(R.cur ^ 1) * d->W;
        const uint32_t k = d->condmap[nfa_cond(R.prev, (int)c)];
        R.dead = !nfa_big_step(pool, d, S, N, R.lo, R.hi, k, nfa_interval(pool, d, r));
        R.cur ^= 1;
        R.prev = (r == '\n' ? NP_NL : 0u) | (r < 128 && nfa_word_byte(r) ? NP_WORD : 0u);
        return;
    }
    const uint32_t W = d->W, nivl = d->nivl;
    const uint64_t *T = (const uint64_t *)(pool + d->t_off);
    const uint32_t *ivl = (const uint32_t *)(pool + d->ivl_off);
    const uint64_t *B = (const uint64_t *)(pool + d->b_off);
    const uint16_t *ascii = (const uint16_t *)(pool + d->ascii_off);
    const uint32_t k = d->condmap[nfa_cond(R.prev, (int)c)];
    uint32_t iv;
    if (r < 128) {
        iv = ascii[r];
    } else {  // last interval starting at or below r
        uint32_t lo = 0, hi = nivl;
        while (hi - lo > 1) {
            const uint32_t mid = (lo + hi) >> 1;
            if (ivl[mid] <= r) lo = mid;
            else hi = mid;
        }
        iv = lo;
    }
    uint64_t N[kNfaMaxWords];
#pragma unroll
    for (int u = 0; u < kNfaMaxWords; u++) N[u] = 0;
#pragma unroll
    for (int w = 0; w < kNfaMaxWords; w++) {
        if ((uint32_t)w >= W) break;
        uint64_t x = R.S[w];
        while (x) {
            const uint32_t j = (uint32_t)__builtin_ctzll(x) >> 3;
            const uint32_t v = (uint32_t)(x >> (8 * j)) & 0xFF;
            x &= ~(0xFFull << (8 * j));
            const uint64_t *row = T + (((uint64_t)k * 8 * W + 8 * (uint32_t)w + j) * 256 + v) * W;
#pragma unroll
            for (int u = 0; u < kNfaMaxWords; u++)
                if ((uint32_t)u < W) N[u] |= row[u];
        }
    }
    uint64_t any = 0;
#pragma unroll
    for (int u = 0; u < kNfaMaxWords; u++) {
        if ((uint32_t)u < W) N[u] &= B[(uint64_t)iv * W + u];
        R.S[u] = N[u];
        any |= N[u];
    }
    R.dead = !any;
    R.prev = (r == '\n' ? NP_NL : 0u) | (r < 128 && nfa_word_byte(r) ? NP_WORD : 0u);
}

L7_NFA_INL bool nfa_end(const uint8_t *pool, uint64_t off, const NfaRun &R) {
    if (R.dead) return false;
    const DevNfa *d = (const DevNfa *)(pool + off);
    const uint32_t W = d->W;
    if (W > (uint32_t)kNfaMaxWords)
        return R.big && nfa_big_accepts(pool, d, R.big + (size_t)R.cur * W, R.lo, R.hi, d->condmap[nfa_cond(R.prev, -1)]);
    const uint64_t *Acc = (const uint64_t *)(pool + d->acc_off);
    const uint32_t k = d->condmap[nfa_cond(R.prev, -1)];
    uint64_t hit = 0;
#pragma unroll
    for (int u = 0; u < kNfaMaxWords; u++)
        if ((uint32_t)u < W) hit |= R.S[u] & Acc[(uint64_t)k * W + u];
    return hit != 0;
}

// A large NFA over s[0, n) with its state sets in scratch (2 W words).
L7_HD inline bool nfa_run_big(const uint8_t *pool, const DevNfa *d, const uint8_t *s, uint32_t n, uint64_t *scratch) {
    uint64_t *S = scratch, *N = scratch + d->W;
    S[0] = 1;  // the virtual start position
    uint32_t lo = 0, hi = 0, prev = NP_START;
    for (uint32_t i = 0; i < n;) {
        const uint32_t c = s[i];
        uint32_t width;
        const uint32_t r = nfa_decode(s, i, n, &width);
        if (!nfa_big_step(pool, d, S, N, lo, hi, d->condmap[nfa_cond(prev, (int)c)], nfa_interval(pool, d, r)))
            return false;
        uint64_t *t = S;
        S = N;
        N = t;
        prev = (r == '\n' ? NP_NL : 0u) | (r < 128 && nfa_word_byte(r) ? NP_WORD : 0u);
        i += width;
    }
    return nfa_big_accepts(pool, d, S, lo, hi, d->condmap[nfa_cond(prev, -1)]);
}

// Run the NFA at pool + off over s[0, n); true = accepted.  scratch: 2 W
// words for a large NFA (W > kNfaMaxWords); the launchers give every lane its
// own whenever the pool holds one.
L7_HD inline bool nfa_run(const uint8_t *pool, uint64_t off, const uint8_t *s, uint32_t n, uint64_t *scratch = nullptr) {
    const DevNfa *d = (const DevNfa *)(pool + off);
    if (d->W > (uint32_t)kNfaMaxWords) return scratch && nfa_run_big(pool, d, s, n, scratch);
    const uint32_t W = d->W, nivl = d->nivl;
    const uint64_t *T = (const uint64_t *)(pool + d->t_off);
    const uint32_t *ivl = (const uint32_t *)(pool + d->ivl_off);
    const uint64_t *B = (const uint64_t *)(pool + d->b_off);
    const uint16_t *ascii = (const uint16_t *)(pool + d->ascii_off);
    const uint64_t *Acc = (const uint64_t *)(pool + d->acc_off);
    uint64_t S[kNfaMaxWords];
#pragma unroll
    for (int w = 0; w < kNfaMaxWords; w++) S[w] = w == 0 ? 1 : 0;  // the virtual start position
    uint32_t prev = NP_START;
    for (uint32_t i = 0; i < n;) {
        const uint32_t c = s[i];
        uint32_t width;
        const uint32_t r = nfa_decode(s, i, n, &width);
        const uint32_t k = d->condmap[nfa_cond(prev, (int)c)];
        uint32_t iv;
        if (r < 128) {
            iv = ascii[r];
        } else {  // last interval starting at or below r
            uint32_t lo = 0, hi = nivl;
            while (hi - lo > 1) {
                const uint32_t mid = (lo + hi) >> 1;
                if (ivl[mid] <= r) lo = mid;
                else hi = mid;
            }
            iv = lo;
        }
        uint64_t N[kNfaMaxWords];
#pragma unroll
        for (int u = 0; u < kNfaMaxWords; u++) N[u] = 0;
#pragma unroll
        for (int w = 0; w < kNfaMaxWords; w++) {
            if ((uint32_t)w >= W) break;
            uint64_t x = S[w];
            while (x) {
                const uint32_t j = (uint32_t)__builtin_ctzll(x) >> 3;
                const uint32_t v = (uint32_t)(x >> (8 * j)) & 0xFF;
                x &= ~(0xFFull << (8 * j));
                const uint64_t *row = T + (((uint64_t)k * 8 * W + 8 * (uint32_t)w + j) * 256 + v) * W;
#pragma unroll
                for (int u = 0; u < kNfaMaxWords; u++)
                    if ((uint32_t)u < W) N[u] |= row[u];
            }
        }
        uint64_t any = 0;
#pragma unroll
        for (int u = 0; u < kNfaMaxWords; u++) {
            if ((uint32_t)u < W) N[u] &= B[(uint64_t)iv * W + u];
            S[u] = N[u];
            any |= N[u];
        }
        if (!any) return false;
        prev = (r == '\n' ? NP_NL : 0u) | (r < 128 && nfa_word_byte(r) ? NP_WORD : 0u);
        i += width;
    }
    const uint32_t k = d->condmap[nfa_cond(prev, -1)];
    uint64_t hit = 0;
#pragma unroll
    for (int u = 0; u < kNfaMaxWords; u++)
        if ((uint32_t)u < W) hit |= S[u] & Acc[(uint64_t)k * W + u];
    return hit != 0;
}

}  // namespace l7
