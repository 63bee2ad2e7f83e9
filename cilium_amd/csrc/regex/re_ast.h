// Go regexp/syntax-compatible AST for the L7 rule compiler (product code).
//
// Semantics follow Go 1.10.3 regexp/syntax with syntax.Perl flags, which is
// what the reference validates HTTP rules with (pkg/policy/api/http.go:66-84)
// and evaluates proxylib key/file/table regexes with
// (proxylib/memcached/parser.go:89-95, proxylib/r2d2/r2d2parser.go:103).
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace l7 {
namespace re {

// Inclusive rune ranges, kept sorted and merged ("clean").
struct RuneSet {
    std::vector<std::pair<int32_t, int32_t>> r;
    void add(int32_t lo, int32_t hi) { r.emplace_back(lo, hi); }
    void clean();
    void negate();  // complement within [0, 0x10FFFF]; requires clean
    bool contains(int32_t c) const;
    bool empty() const { return r.empty(); }
};

enum class Op : uint8_t {
    NoMatch, Empty, Class, AnyNotNL, Any,
    BeginLine, EndLine, BeginText, EndText, WordBoundary, NoWordBoundary,
    Star, Plus, Quest, Repeat, Concat, Alternate,
    // raw-byte ops, built by the rule compiler for Envoy exact/prefix/suffix
    // matchers (byte equality, not rune semantics); never produced by Parse
    ByteString, AnyBytes,
    // parser-internal pseudo ops
    LeftParen = 100, VerticalBar,
};

struct Node {
    Op op;
    int flags = 0;
    int min = 0, max = 0;
    RuneSet cls;
    std::string bytes;  // ByteString
    std::vector<std::unique_ptr<Node>> sub;
    explicit Node(Op o, int f = 0) : op(o), flags(f) {}
};

// Parse `pat` with Go's syntax.Perl flags.  On failure returns nullptr and
// sets `err` to Go's message: "error parsing regexp: <code>: `<expr>`".
std::unique_ptr<Node> Parse(const std::string &pat, std::string *err);

// Unicode helpers shared by parser and NFA builder.
int32_t SimpleFold(int32_t r);
// Go utf8.DecodeRune; returns width (0 at end), sets *r (0xFFFD on error).
int DecodeRune(const uint8_t *s, size_t n, int32_t *r);

}  // namespace re
}  // namespace l7
