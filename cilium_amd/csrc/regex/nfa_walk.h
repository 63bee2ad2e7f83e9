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

// Streaming walk (for text the caller produces rune by rune, e.g. the
// lowered cassandra table name): nfa_begin, one nfa_step per rune (r, and c =
// the first byte of its encoding, which the empty-width conditions look at),
// nfa_end.  Same step as nfa_run below, which keeps its own loop so its state
// stays in registers in the pre-pass kernels.
struct NfaRun {
    uint64_t S[kNfaMaxWords];
    uint32_t prev;
    bool dead;
};

L7_NFA_INL void nfa_begin(NfaRun &R) {
#pragma unroll
    for (int w = 0; w < kNfaMaxWords; w++) R.S[w] = w == 0 ? 1 : 0;  // the virtual start position
    R.prev = NP_START;
    R.dead = false;
}

L7_NFA_INL void nfa_step(const uint8_t *pool, uint64_t off, NfaRun &R, uint32_t r, uint32_t c) {
    if (R.dead) return;
    const DevNfa *d = (const DevNfa *)(pool + off);
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
    const uint64_t *Acc = (const uint64_t *)(pool + d->acc_off);
    const uint32_t k = d->condmap[nfa_cond(R.prev, -1)];
    uint64_t hit = 0;
#pragma unroll
    for (int u = 0; u < kNfaMaxWords; u++)
        if ((uint32_t)u < W) hit |= R.S[u] & Acc[(uint64_t)k * W + u];
    return hit != 0;
}

// Run the NFA at pool + off over s[0, n); true = accepted.
L7_HD inline bool nfa_run(const uint8_t *pool, uint64_t off, const uint8_t *s, uint32_t n) {
    const DevNfa *d = (const DevNfa *)(pool + off);
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
