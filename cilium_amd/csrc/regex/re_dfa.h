// Multi-pattern byte DFA compiler for Go-syntax regexps (product code).
//
// Patterns are Go regexps (re_ast.h).  The DFA runs over raw bytes but
// reproduces Go's rune semantics exactly: input is decoded like
// utf8.DecodeRune (an invalid byte is U+FFFD of width 1), so the NFA carries a
// small "guard" per thread for bytes consumed as invalid lead bytes (the guess
// is killed if the following bytes turn out to complete a valid sequence).
// Empty-width assertions (^ $ \A \z \b \B, (?m)^ $) are resolved with the
// previous-byte context kept in the DFA state.
//
// Each pattern is either anchored (full match: regexp "^(?:p)$", the HTTP
// header contract, envoy HeaderUtility regex_match) or unanchored (Go
// regexp.Match, the proxylib contract).  The DFA reports, per state, the set
// of patterns that accept if the input ends there.
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "re_ast.h"

namespace l7 {
namespace re {

struct Pattern {
    const Node *ast;
    bool anchored;
};

struct DFA {
    int nstates = 0;        // state 0 is the dead state
    int ncls = 0;
    int start = 0;
    uint8_t cls[256] = {0};
    std::vector<uint16_t> next;                 // [nstates][ncls]
    std::vector<std::vector<uint64_t>> accept;  // per state: bitset over pattern index (EOF acceptance)
    int npatterns = 0;
    bool absorbing(int s) const;                // every transition loops back to s
};

// Returns false (and sets *err) when the determinised automaton would exceed
// max_states; callers split the pattern set and retry.
bool BuildDFA(const std::vector<Pattern> &pats, int max_states, DFA *out, std::string *err);

// Bit-parallel Glushkov automaton of ONE pattern, over runes: the fallback
// for a pattern whose DFA alone exceeds the state budget (its NFA has few
// positions even when the subset construction explodes, e.g.
// (a|b)*a(a|b){14}).
//
// Positions are the pattern's rune-class occurrences (one per class, however
// many UTF-8 sequences it spans); position 0 is the virtual start.  The input
// is decoded like utf8.DecodeRune (an invalid byte is U+FFFD of width 1), so
// Go's rune semantics need no byte-level guards here.  A state set S is a
// bitset over positions; reading rune r at the boundary whose empty-width
// condition class is k:
//     S' = Follow_k(S) & B[interval of r]
// where Follow_k(p) is every position reachable from p through the epsilon
// closure under k, and B[iv] the positions whose class holds the rune
// interval iv.  The input is accepted iff S & Acc_k(end) != 0.
//
// A small automaton (W <= dense_words) keeps Follow_k as dense rows; a large
// one (up to max_positions, e.g. .{1000}x.{1000}: 2,003 positions) as sparse
// rows: Follow_k(p) = the (word, mask) pairs of its non-zero words, shared by
// the positions whose epsilon closures coincide.
struct BitNfa {
    int m = 0;                    // positions (incl. the virtual start)
    int W = 0;                    // u64 words per state set
    int K = 0;                    // empty-width condition classes
    uint8_t condmap[64] = {0};    // NC_* condition bits (nfa_walk.h) -> class
    std::vector<uint64_t> follow; // dense: [K][m][W]
    bool sparse = false;
    std::vector<uint32_t> row_of;   // sparse: [K][m] -> row
    std::vector<uint32_t> row_ptr;  // sparse: [rows + 1] -> first pair
    std::vector<uint32_t> pair_w;   // sparse: word of each pair
    std::vector<uint64_t> pair_m;   // sparse: mask of each pair
    std::vector<uint64_t> acc;    // [K][W]
    std::vector<int32_t> ivl_lo;  // rune intervals [ivl_lo[i], ivl_lo[i+1]) (last ends at 0x110000)
    std::vector<uint64_t> b;      // [interval][W]
};
// false (and *err) when the pattern needs more than max_positions positions.
bool BuildBitNfa(const Pattern &p, int max_positions, BitNfa *out, std::string *err, int dense_words = 16);

// Reference walk over the compiled tables (used by tests and by the host-side
// table validator; the product's matching runs on the GPU).
std::vector<uint64_t> RunDFA(const DFA &d, const uint8_t *s, size_t n);

}  // namespace re
}  // namespace l7
