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

// Reference walk over the compiled tables (used by tests and by the host-side
// table validator; the product's matching runs on the GPU).
std::vector<uint64_t> RunDFA(const DFA &d, const uint8_t *s, size_t n);

}  // namespace re
}  // namespace l7
