// Go regexp/syntax parser (syntax.Perl flags) for the L7 rule compiler.
//
// Reproduces the accept/reject set and error texts of Go 1.10.3
// regexp/syntax.Parse, because a rule the reference rejects in
// PortRuleHTTP.Sanitize (pkg/policy/api/http.go:66-84) must be rejected here
// too (KAT: pkg/policy/api/rule_validation_test.go:155-205, `*` is an error).
// The grammar is Go's operator-stack algorithm: repetition applies to the top
// of the stack, `|` and `)` collapse it, `(?flags)` changes flags for the rest
// of the enclosing group.
#include <algorithm>
#include <cstring>

#include "re_ast.h"
#include "unicode_tables.h"

namespace l7 {
namespace re {

static constexpr int32_t kMaxRune = 0x10FFFF;
static constexpr int32_t kRuneError = 0xFFFD;

enum : int { kFold = 1, kDotNL = 2, kOneLine = 4, kNonGreedy = 8 };

int DecodeRune(const uint8_t *s, size_t n, int32_t *r) {
    if (n == 0) { *r = kRuneError; return 0; }
    uint8_t b0 = s[0];
    if (b0 < 0x80) { *r = b0; return 1; }
    int sz;
    uint8_t lo = 0x80, hi = 0xBF;
    if (b0 >= 0xC2 && b0 <= 0xDF) sz = 2;
    else if (b0 >= 0xE0 && b0 <= 0xEF) { sz = 3; if (b0 == 0xE0) lo = 0xA0; else if (b0 == 0xED) hi = 0x9F; }
    else if (b0 >= 0xF0 && b0 <= 0xF4) { sz = 4; if (b0 == 0xF0) lo = 0x90; else if (b0 == 0xF4) hi = 0x8F; }
    else { *r = kRuneError; return 1; }
    if (n < (size_t)sz || s[1] < lo || s[1] > hi) { *r = kRuneError; return 1; }
    if (sz == 2) { *r = ((b0 & 0x1F) << 6) | (s[1] & 0x3F); return 2; }
    if (s[2] < 0x80 || s[2] > 0xBF) { *r = kRuneError; return 1; }
    if (sz == 3) { *r = ((b0 & 0x0F) << 12) | ((s[1] & 0x3F) << 6) | (s[2] & 0x3F); return 3; }
    if (s[3] < 0x80 || s[3] > 0xBF) { *r = kRuneError; return 1; }
    *r = ((b0 & 0x07) << 18) | ((s[1] & 0x3F) << 12) | ((s[2] & 0x3F) << 6) | (s[3] & 0x3F);
    return 4;
}

int32_t SimpleFold(int32_t r) {
    const auto *b = UNI_FOLD_PAIRS, *e = UNI_FOLD_PAIRS + UNI_FOLD_NPAIRS;
    auto it = std::lower_bound(b, e, (uint32_t)r, [](const uint32_t p[2], uint32_t v) { return p[0] < v; });
    if (it != e && (int32_t)(*it)[0] == r) return (int32_t)(*it)[1];
    return r;
}

void RuneSet::clean() {
    if (r.empty()) return;
    std::sort(r.begin(), r.end());
    std::vector<std::pair<int32_t, int32_t>> o;
    for (auto &p : r) {
        if (!o.empty() && p.first <= o.back().second + 1) o.back().second = std::max(o.back().second, p.second);
        else o.push_back(p);
    }
    r.swap(o);
}
void RuneSet::negate() {
    std::vector<std::pair<int32_t, int32_t>> o;
    int32_t next = 0;
    for (auto &p : r) {
        if (p.first > next) o.emplace_back(next, p.first - 1);
        next = p.second + 1;
    }
    if (next <= kMaxRune) o.emplace_back(next, kMaxRune);
    r.swap(o);
}
bool RuneSet::contains(int32_t c) const {
    auto it = std::upper_bound(r.begin(), r.end(), std::make_pair(c, INT32_MAX));
    if (it == r.begin()) return false;
    --it;
    return c >= it->first && c <= it->second;
}

// appendFoldedRange: each rune in [lo,hi] plus its simple-fold orbit.
static void AddFolded(RuneSet &s, int32_t lo, int32_t hi) {
    s.add(lo, hi);
    const auto *b = UNI_FOLD_PAIRS, *e = UNI_FOLD_PAIRS + UNI_FOLD_NPAIRS;
    auto it = std::lower_bound(b, e, (uint32_t)lo, [](const uint32_t p[2], uint32_t v) { return p[0] < v; });
    for (; it != e && (int32_t)(*it)[0] <= hi; ++it) {
        int32_t r0 = (int32_t)(*it)[0];
        for (int32_t f = SimpleFold(r0); f != r0; f = SimpleFold(f)) s.add(f, f);
    }
}
static void AppendClass(RuneSet &dst, const RuneSet &src, bool fold, bool negate) {
    RuneSet t;
    for (auto &p : src.r) { if (fold) AddFolded(t, p.first, p.second); else t.add(p.first, p.second); }
    t.clean();
    if (negate) t.negate();
    dst.r.insert(dst.r.end(), t.r.begin(), t.r.end());
}

namespace {

struct Group { const char *name; int sign; std::vector<std::pair<int32_t, int32_t>> ranges; };

const std::vector<Group> &PerlGroups() {
    static const std::vector<Group> g = {
        {"\\d", 1, {{'0', '9'}}}, {"\\D", -1, {{'0', '9'}}},
        {"\\s", 1, {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}}, {"\\S", -1, {{'\t', '\n'}, {'\f', '\r'}, {' ', ' '}}},
        {"\\w", 1, {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}}, {"\\W", -1, {{'0', '9'}, {'A', 'Z'}, {'_', '_'}, {'a', 'z'}}},
    };
    return g;
}
const std::vector<Group> &PosixGroups() {
    static const std::vector<Group> g = [] {
        std::vector<std::pair<const char *, std::vector<std::pair<int32_t, int32_t>>>> base = {
            {"alnum", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}}}, {"alpha", {{'A', 'Z'}, {'a', 'z'}}},
            {"ascii", {{0, 0x7F}}}, {"blank", {{'\t', '\t'}, {' ', ' '}}}, {"cntrl", {{0, 0x1F}, {0x7F, 0x7F}}},
            {"digit", {{'0', '9'}}}, {"graph", {{'!', '~'}}}, {"lower", {{'a', 'z'}}}, {"print", {{' ', '~'}}},
            {"punct", {{'!', '/'}, {':', '@'}, {'[', '`'}, {'{', '~'}}}, {"space", {{'\t', '\r'}, {' ', ' '}}},
            {"upper", {{'A', 'Z'}}}, {"word", {{'0', '9'}, {'A', 'Z'}, {'a', 'z'}, {'_', '_'}}},
            {"xdigit", {{'0', '9'}, {'A', 'F'}, {'a', 'f'}}},
        };
        std::vector<Group> out;
        static std::vector<std::string> names;
        names.reserve(64);
        for (auto &b : base) {
            names.push_back(std::string("[:") + b.first + ":]");
            out.push_back({nullptr, 1, b.second});
            names.push_back(std::string("[:^") + b.first + ":]");
            out.push_back({nullptr, -1, b.second});
        }
        for (size_t i = 0; i < out.size(); i++) out[i].name = names[i].c_str();
        return out;
    }();
    return g;
}

bool IsAlnum(int32_t c) { return (c >= '0' && c <= '9') || (c >= 'A' && c <= 'Z') || (c >= 'a' && c <= 'z'); }
int Unhex(int32_t c) {
    if (c >= '0' && c <= '9') return c - '0';
    if (c >= 'a' && c <= 'f') return c - 'a' + 10;
    if (c >= 'A' && c <= 'F') return c - 'A' + 10;
    return -1;
}

class Parser {
public:
    explicit Parser(const std::string &s) : s_(s) {}
    std::unique_ptr<Node> Run(std::string *err);

private:
    const std::string &s_;
    std::vector<std::unique_ptr<Node>> st_;
    int flags_ = kOneLine;  // syntax.Perl = ClassNL|OneLine|PerlX|UnicodeGroups
    std::string err_;

    bool Fail(const char *code, size_t pos, size_t len) {
        if (err_.empty()) err_ = std::string("error parsing regexp: ") + code + ": `" + s_.substr(pos, len) + "`";
        return false;
    }
    size_t n() const { return s_.size(); }
    uint8_t at(size_t i) const { return (uint8_t)s_[i]; }
    // nextRune: returns width or -1 on invalid UTF-8 (error set)
    int Next(size_t i, int32_t *r) {
        int w = DecodeRune((const uint8_t *)s_.data() + i, n() - i, r);
        if (*r == kRuneError && w == 1) { Fail("invalid UTF-8", i, n() - i); return -1; }
        return w;
    }
    void Push(std::unique_ptr<Node> x) { st_.push_back(std::move(x)); }
    void Literal(int32_t r) {
        auto x = std::make_unique<Node>(Op::Class, flags_);
        if (flags_ & kFold) AddFolded(x->cls, r, r); else x->cls.add(r, r);
        x->cls.clean();
        Push(std::move(x));
    }
    void Concat();
    void Alternate();
    bool Repeat(Op op, int mn, int mx, size_t before, size_t *after, size_t lastrep, bool haslast);
    int Escape(size_t i, int32_t *out);  // returns consumed or -1
    int PerlClass(size_t i, RuneSet &dst);
    int NamedClass(size_t i, RuneSet &dst);
    int UnicodeClass(size_t i, RuneSet &dst);
    int Class(size_t i);
    int PerlFlags(size_t i);
    bool RightParen();
    void AppendGroup(RuneSet &dst, const Group &g) {
        RuneSet src; for (auto &p : g.ranges) src.add(p.first, p.second);
        AppendClass(dst, src, (flags_ & kFold) != 0, g.sign < 0);
    }
};

void Parser::Concat() {
    size_t i = st_.size();
    while (i > 0 && st_[i - 1]->op < Op::LeftParen) i--;
    size_t cnt = st_.size() - i;
    std::unique_ptr<Node> c;
    if (cnt == 0) c = std::make_unique<Node>(Op::Empty, flags_);
    else if (cnt == 1) c = std::move(st_[i]);
    else {
        c = std::make_unique<Node>(Op::Concat, flags_);
        for (size_t k = i; k < st_.size(); k++) c->sub.push_back(std::move(st_[k]));
    }
    st_.resize(i);
    Push(std::move(c));
}

void Parser::Alternate() {
    size_t i = st_.size();
    while (i > 0 && st_[i - 1]->op != Op::LeftParen) i--;
    std::vector<std::unique_ptr<Node>> alts;
    for (size_t k = i; k < st_.size(); k++) if (st_[k]->op != Op::VerticalBar) alts.push_back(std::move(st_[k]));
    st_.resize(i);
    if (alts.size() == 1) { Push(std::move(alts[0])); return; }
    auto a = std::make_unique<Node>(Op::Alternate, flags_);
    a->sub = std::move(alts);
    Push(std::move(a));
}

static bool RepeatIsValid(const Node *re, int n) {
    if (re->op == Op::Repeat) {
        int m = re->max;
        if (m == 0) return true;
        if (m < 0) m = re->min;
        if (m > n) return false;
        if (m > 0) n /= m;
    }
    for (auto &s : re->sub) if (!RepeatIsValid(s.get(), n)) return false;
    return true;
}

// syntax.(*parser).repeat.  `before` is the operator's offset, *after the
// offset just past it; lastrep is the offset of the previous repetition op.
bool Parser::Repeat(Op op, int mn, int mx, size_t before, size_t *after, size_t lastrep, bool haslast) {
    size_t a = *after;
    if (a < n() && at(a) == '?') a++;  // non-greedy: same language
    if (haslast) return Fail("invalid nested repetition operator", lastrep, a - lastrep);
    if (st_.empty() || st_.back()->op >= Op::LeftParen) return Fail("missing argument to repetition operator", before, a - before);
    auto x = std::make_unique<Node>(op, flags_);
    x->min = mn; x->max = mx;
    x->sub.push_back(std::move(st_.back()));
    st_.back() = std::move(x);
    if (op == Op::Repeat && (mn >= 2 || mx >= 2) && !RepeatIsValid(st_.back().get(), 1000))
        return Fail("invalid repeat count", before, a - before);
    *after = a;
    return true;
}

int Parser::Escape(size_t i0, int32_t *out) {
    size_t i = i0 + 1;
    if (i >= n()) { Fail("trailing backslash at end of expression", 0, 0); return -1; }
    int32_t c;
    int w = Next(i, &c);
    if (w < 0) return -1;
    i += w;
    switch (c) {
    case '1': case '2': case '3': case '4': case '5': case '6': case '7':
        if (i >= n() || at(i) < '0' || at(i) > '7') break;
        [[fallthrough]];
    case '0': {
        int32_t r = c - '0';
        for (int k = 1; k < 3; k++) {
            if (i >= n() || at(i) < '0' || at(i) > '7') break;
            r = r * 8 + (at(i) - '0');
            i++;
        }
        *out = r;
        return (int)(i - i0);
    }
    case 'x': {
        if (i >= n()) break;
        w = Next(i, &c); if (w < 0) return -1; i += w;
        if (c == '{') {
            int nhex = 0; int32_t r = 0;
            for (;;) {
                if (i >= n()) goto bad;
                w = Next(i, &c); if (w < 0) return -1; i += w;
                if (c == '}') break;
                int v = Unhex(c);
                if (v < 0) goto bad;
                r = r * 16 + v;
                if (r > kMaxRune) goto bad;
                nhex++;
            }
            if (nhex == 0) goto bad;
            *out = r;
            return (int)(i - i0);
        }
        int x = Unhex(c);
        int32_t c2;
        w = Next(i, &c2); if (w < 0) return -1; i += w;
        int y = Unhex(c2);
        if (x < 0 || y < 0) break;
        *out = x * 16 + y;
        return (int)(i - i0);
    }
    case 'a': *out = 7; return (int)(i - i0);
    case 'f': *out = 12; return (int)(i - i0);
    case 'n': *out = 10; return (int)(i - i0);
    case 'r': *out = 13; return (int)(i - i0);
    case 't': *out = 9; return (int)(i - i0);
    case 'v': *out = 11; return (int)(i - i0);
    default:
        if (c < 0x80 && !IsAlnum(c)) { *out = c; return (int)(i - i0); }
        break;
    }
bad:
    Fail("invalid escape sequence", i0, i - i0);
    return -1;
}

int Parser::PerlClass(size_t i, RuneSet &dst) {
    if (n() - i < 2 || at(i) != '\\') return 0;
    for (auto &g : PerlGroups())
        if ((uint8_t)g.name[1] == at(i + 1)) { AppendGroup(dst, g); return 2; }
    return 0;
}

int Parser::NamedClass(size_t i, RuneSet &dst) {
    if (n() - i < 2 || at(i) != '[' || at(i + 1) != ':') return 0;
    size_t e = s_.find(":]", i + 2);
    if (e == std::string::npos) return 0;
    size_t len = e + 2 - i;
    for (auto &g : PosixGroups())
        if (strlen(g.name) == len && s_.compare(i, len, g.name) == 0) { AppendGroup(dst, g); return (int)len; }
    Fail("invalid character class range", i, len);
    return -1;
}

int Parser::UnicodeClass(size_t i, RuneSet &dst) {
    if (n() - i < 2 || at(i) != '\\' || (at(i + 1) != 'p' && at(i + 1) != 'P')) return 0;
    int sign = at(i + 1) == 'P' ? -1 : 1;
    int32_t c;
    int w = DecodeRune((const uint8_t *)s_.data() + i + 2, n() - i - 2, &c);
    if (c == kRuneError && w == 1) { Fail("invalid UTF-8", i + 2, n() - i - 2); return -1; }
    std::string name;
    size_t seqlen;
    if (c != '{') {
        seqlen = 2 + w;
        name = s_.substr(i + 2, w);
    } else {
        size_t e = s_.find('}', i);
        if (e == std::string::npos) { Fail("invalid character class range", i, n() - i); return -1; }
        seqlen = e + 1 - i;
        name = s_.substr(i + 3, e - i - 3);
    }
    if (!name.empty() && name[0] == '^') { sign = -sign; name.erase(0, 1); }
    RuneSet tab;
    bool fold = false;
    if (name == "Any") {
        tab.add(0, kMaxRune);
    } else {
        const uni_table_t *t = nullptr;
        for (int k = 0; k < UNI_NTABLES; k++) if (name == UNI_TABLES[k].name) { t = &UNI_TABLES[k]; break; }
        if (!t) { Fail("invalid character class range", i, seqlen); return -1; }
        for (int k = 0; k < t->n; k++) tab.add((int32_t)UNI_RANGES[t->off + k][0], (int32_t)UNI_RANGES[t->off + k][1]);
        // Go carries fold tables only for these (unicode.FoldCategory / FoldScript)
        static const char *kFoldNames[] = {"L", "Ll", "Lt", "Lu", "M", "Mn", "Common", "Greek", "Inherited"};
        for (auto *f : kFoldNames) if (name == f) fold = true;
    }
    AppendClass(dst, tab, (flags_ & kFold) && fold, sign < 0);
    return (int)seqlen;
}

int Parser::Class(size_t i0) {
    size_t i = i0 + 1;
    auto x = std::make_unique<Node>(Op::Class, flags_);
    int sign = 1;
    if (i < n() && at(i) == '^') { sign = -1; i++; }
    bool first = true;
    while (i >= n() || at(i) != ']' || first) {
        first = false;
        int k;
        if (n() - i > 2 && at(i) == '[' && at(i + 1) == ':') {
            k = NamedClass(i, x->cls);
            if (k < 0) return -1;
            if (k > 0) { i += k; continue; }
        }
        k = UnicodeClass(i, x->cls);
        if (k < 0) return -1;
        if (k > 0) { i += k; continue; }
        k = PerlClass(i, x->cls);
        if (k > 0) { i += k; continue; }
        size_t rs = i;
        int32_t lo, hi;
        if (i >= n()) { Fail("missing closing ]", i0, n() - i0); return -1; }
        if (at(i) == '\\') { k = Escape(i, &lo); if (k < 0) return -1; i += k; }
        else { k = Next(i, &lo); if (k < 0) return -1; i += k; }
        hi = lo;
        if (n() - i >= 2 && at(i) == '-' && at(i + 1) != ']') {
            i++;
            if (at(i) == '\\') { k = Escape(i, &hi); if (k < 0) return -1; i += k; }
            else { k = Next(i, &hi); if (k < 0) return -1; i += k; }
            if (hi < lo) { Fail("invalid character class range", rs, i - rs); return -1; }
        }
        if (flags_ & kFold) AddFolded(x->cls, lo, hi); else x->cls.add(lo, hi);
    }
    i++;
    x->cls.clean();
    if (sign < 0) x->cls.negate();
    Push(std::move(x));
    return (int)(i - i0);
}

int Parser::PerlFlags(size_t i0) {
    if (n() - i0 > 4 && at(i0 + 2) == 'P' && at(i0 + 3) == '<') {
        size_t e = s_.find('>', i0);
        if (e == std::string::npos) { Fail("invalid named capture", i0, n() - i0); return -1; }
        bool ok = e > i0 + 4;
        for (size_t k = i0 + 4; k < e; k++) if (!(at(k) == '_' || IsAlnum(at(k)))) ok = false;
        if (!ok) { Fail("invalid named capture", i0, e + 1 - i0); return -1; }
        Push(std::make_unique<Node>(Op::LeftParen, flags_));
        return (int)(e + 1 - i0);
    }
    size_t i = i0 + 2;
    int fl = flags_, sign = 1;
    bool saw = false;
    while (i < n()) {
        int32_t c;
        int w = Next(i, &c);
        if (w < 0) return -1;
        i += w;
        switch (c) {
        case 'i': fl |= kFold; saw = true; continue;
        case 'm': fl &= ~kOneLine; saw = true; continue;
        case 's': fl |= kDotNL; saw = true; continue;
        case 'U': fl |= kNonGreedy; saw = true; continue;
        case '-':
            if (sign < 0) break;
            sign = -1; fl = ~fl; saw = false;
            continue;
        case ':': case ')':
            if (sign < 0) { if (!saw) break; fl = ~fl; }
            if (c == ':') Push(std::make_unique<Node>(Op::LeftParen, flags_));
            flags_ = fl;
            return (int)(i - i0);
        default:
            break;
        }
        break;
    }
    Fail("invalid or unsupported Perl syntax", i0, i - i0);
    return -1;
}

bool Parser::RightParen() {
    Concat();
    Alternate();
    size_t k = st_.size();
    if (k < 2 || st_[k - 2]->op != Op::LeftParen) return Fail("unexpected )", 0, n());
    auto re1 = std::move(st_[k - 1]);
    flags_ = st_[k - 2]->flags;
    st_.resize(k - 2);
    Push(std::move(re1));
    return true;
}

static bool ParseInt(const std::string &s, size_t *i, int *v) {
    size_t st = *i;
    if (st >= s.size() || s[st] < '0' || s[st] > '9') return false;
    if (s.size() - st >= 2 && s[st] == '0' && s[st + 1] >= '0' && s[st + 1] <= '9') return false;
    size_t e = st;
    while (e < s.size() && s[e] >= '0' && s[e] <= '9') e++;
    long x = 0;
    for (size_t k = st; k < e; k++) { if (x >= 100000000) { x = -1; break; } x = x * 10 + (s[k] - '0'); }
    *v = (int)x;
    *i = e;
    return true;
}
// parseRepeat on s[i] == '{'; returns end offset or 0
static size_t ParseRepeat(const std::string &s, size_t i, int *mn, int *mx) {
    if (i >= s.size() || s[i] != '{') return 0;
    size_t k = i + 1;
    if (!ParseInt(s, &k, mn)) return 0;
    if (k >= s.size()) return 0;
    if (s[k] != ',') *mx = *mn;
    else {
        k++;
        if (k >= s.size()) return 0;
        if (s[k] == '}') *mx = -1;
        else {
            if (!ParseInt(s, &k, mx)) return 0;
            if (*mx < 0) *mn = -1;
        }
    }
    if (k >= s.size() || s[k] != '}') return 0;
    return k + 1;
}

std::unique_ptr<Node> Parser::Run(std::string *err) {
    size_t i = 0;
    bool haslast = false;
    size_t lastrep = 0;
    bool ok = true;
    while (ok && i < n()) {
        bool rep = false;
        size_t repat = i;
        uint8_t c = at(i);
        switch (c) {
        case '(':
            if (n() - i >= 2 && at(i + 1) == '?') { int k = PerlFlags(i); if (k < 0) { ok = false; break; } i += k; break; }
            Push(std::make_unique<Node>(Op::LeftParen, flags_));
            i++;
            break;
        case '|':
            Concat();
            Push(std::make_unique<Node>(Op::VerticalBar, flags_));
            i++;
            break;
        case ')':
            if (!RightParen()) { ok = false; break; }
            i++;
            break;
        case '^': Push(std::make_unique<Node>((flags_ & kOneLine) ? Op::BeginText : Op::BeginLine, flags_)); i++; break;
        case '$': Push(std::make_unique<Node>((flags_ & kOneLine) ? Op::EndText : Op::EndLine, flags_)); i++; break;
        case '.': Push(std::make_unique<Node>((flags_ & kDotNL) ? Op::Any : Op::AnyNotNL, flags_)); i++; break;
        case '[': { int k = Class(i); if (k < 0) { ok = false; break; } i += k; break; }
        case '*': case '+': case '?': {
            Op op = c == '*' ? Op::Star : (c == '+' ? Op::Plus : Op::Quest);
            size_t after = i + 1;
            if (!Repeat(op, 0, 0, i, &after, lastrep, haslast)) { ok = false; break; }
            rep = true;
            i = after;
            break;
        }
        case '{': {
            int mn = 0, mx = 0;
            size_t e = ParseRepeat(s_, i, &mn, &mx);
            if (!e) { Literal('{'); i++; break; }
            if (mn < 0 || mn > 1000 || mx > 1000 || (mx >= 0 && mn > mx)) { Fail("invalid repeat count", i, e - i); ok = false; break; }
            size_t after = e;
            if (!Repeat(Op::Repeat, mn, mx, i, &after, lastrep, haslast)) { ok = false; break; }
            rep = true;
            i = after;
            break;
        }
        case '\\': {
            if (n() - i >= 2) {
                uint8_t c1 = at(i + 1);
                if (c1 == 'A') { Push(std::make_unique<Node>(Op::BeginText, flags_)); i += 2; break; }
                if (c1 == 'b') { Push(std::make_unique<Node>(Op::WordBoundary, flags_)); i += 2; break; }
                if (c1 == 'B') { Push(std::make_unique<Node>(Op::NoWordBoundary, flags_)); i += 2; break; }
                if (c1 == 'C') { Fail("invalid escape sequence", i, 2); ok = false; break; }
                if (c1 == 'z') { Push(std::make_unique<Node>(Op::EndText, flags_)); i += 2; break; }
                if (c1 == 'Q') {
                    size_t e = s_.find("\\E", i + 2);
                    size_t litend = e == std::string::npos ? n() : e;
                    size_t adv = e == std::string::npos ? n() : e + 2;
                    size_t j = i + 2;
                    while (ok && j < litend) {
                        int32_t r;
                        int w = DecodeRune((const uint8_t *)s_.data() + j, litend - j, &r);
                        if (r == kRuneError && w == 1) { Fail("invalid UTF-8", j, litend - j); ok = false; break; }
                        Literal(r);
                        j += w;
                    }
                    i = adv;
                    break;
                }
            }
            auto x = std::make_unique<Node>(Op::Class, flags_);
            int k = UnicodeClass(i, x->cls);
            if (k < 0) { ok = false; break; }
            if (k == 0) k = PerlClass(i, x->cls);
            if (k > 0) { x->cls.clean(); Push(std::move(x)); i += k; break; }
            int32_t r;
            k = Escape(i, &r);
            if (k < 0) { ok = false; break; }
            Literal(r);
            i += k;
            break;
        }
        default: {
            int32_t r;
            int w = Next(i, &r);
            if (w < 0) { ok = false; break; }
            Literal(r);
            i += w;
            break;
        }
        }
        haslast = rep;
        lastrep = repat;
    }
    if (ok) {
        Concat();
        Alternate();
        if (st_.size() != 1) { Fail("missing closing )", 0, n()); ok = false; }
    }
    if (!ok) { if (err) *err = err_; return nullptr; }
    return std::move(st_[0]);
}

}  // namespace

std::unique_ptr<Node> Parse(const std::string &pat, std::string *err) {
    Parser p(pat);
    return p.Run(err);
}

}  // namespace re
}  // namespace l7
