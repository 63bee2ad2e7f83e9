// NFA construction + subset construction + minimisation (product code).
// See re_dfa.h for the semantics being reproduced.
#include "re_dfa.h"

#include <algorithm>
#include <cstring>
#include <map>
#include <unordered_map>

namespace l7 {
namespace re {
namespace {

// ---- guards: a byte consumed as an *invalid* UTF-8 lead (U+FFFD width 1)
// is only a correct guess if the following bytes do NOT complete a valid
// sequence for that lead (utf8.DecodeRune).  A guard is the sequence of byte
// ranges that would complete it; the thread dies if they all occur.
enum : uint8_t { G_NONE = 0, G2, G3, G4, GE0, GED, GF0, GF4, G_DIE = 0xFF };
struct GuardInfo { uint8_t lo, hi, residual; };
const GuardInfo kGuard[8] = {
    {1, 0, G_NONE},         // NONE (empty range)
    {0x80, 0xBF, G_DIE},    // G2 : [80-BF]
    {0x80, 0xBF, G2},       // G3 : [80-BF][80-BF]
    {0x80, 0xBF, G3},       // G4 : [80-BF][80-BF][80-BF]
    {0xA0, 0xBF, G2},       // E0 : [A0-BF][80-BF]
    {0x80, 0x9F, G2},       // ED : [80-9F][80-BF]
    {0x90, 0xBF, G3},       // F0 : [90-BF][80-BF][80-BF]
    {0x80, 0x8F, G3},       // F4 : [80-8F][80-BF][80-BF]
};
inline uint8_t GuardStep(uint8_t g, uint8_t b) {
    if (g == G_NONE) return G_NONE;
    const GuardInfo &gi = kGuard[g];
    return (b >= gi.lo && b <= gi.hi) ? gi.residual : G_NONE;
}

// empty-width condition bits
enum : uint8_t { C_BOT = 1, C_EOT = 2, C_BOL = 4, C_EOL = 8, C_WB = 16, C_NWB = 32 };
// previous-byte context kept in DFA states
enum : uint8_t { P_START = 1, P_NL = 2, P_WORD = 4 };

inline bool IsWordByte(int b) {
    return (b >= '0' && b <= '9') || (b >= 'A' && b <= 'Z') || (b >= 'a' && b <= 'z') || b == '_';
}

enum class K : uint8_t { Byte, Split, Assert, Match, Rune /* rune mode: one whole rune of rsets[rset] */ };
struct BTr { uint8_t lo, hi, guard; int to; };
struct NState {
    K k = K::Byte;
    int out = -1, out1 = -1;
    uint8_t cond = 0;
    int acc = -1;   // Match_k / Done_k: pattern id
    int done = -1;  // Match_k of an unanchored pattern: its sticky Done_k state
    int rset = -1;  // K::Rune: its rune class
    std::vector<BTr> tr;
};

int EncLen(int32_t r) { return r < 0x80 ? 1 : r < 0x800 ? 2 : r < 0x10000 ? 3 : 4; }
void Enc(int32_t r, uint8_t *b) {
    switch (EncLen(r)) {
    case 1: b[0] = (uint8_t)r; break;
    case 2: b[0] = (uint8_t)(0xC0 | (r >> 6)); b[1] = (uint8_t)(0x80 | (r & 0x3F)); break;
    case 3: b[0] = (uint8_t)(0xE0 | (r >> 12)); b[1] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); b[2] = (uint8_t)(0x80 | (r & 0x3F)); break;
    default: b[0] = (uint8_t)(0xF0 | (r >> 18)); b[1] = (uint8_t)(0x80 | ((r >> 12) & 0x3F));
             b[2] = (uint8_t)(0x80 | ((r >> 6) & 0x3F)); b[3] = (uint8_t)(0x80 | (r & 0x3F)); break;
    }
}
using Seq = std::vector<std::pair<uint8_t, uint8_t>>;
// Split [lo,hi] into byte-range sequences of valid shortest UTF-8 encodings.
void Utf8Split(int32_t lo, int32_t hi, std::vector<Seq> &out) {
    if (lo > hi) return;
    if (lo <= 0xDFFF && hi >= 0xD800) {  // surrogates never decode as runes
        if (lo < 0xD800) Utf8Split(lo, 0xD7FF, out);
        if (hi > 0xDFFF) Utf8Split(0xE000, hi, out);
        return;
    }
    static const int32_t kMax[] = {0x7F, 0x7FF, 0xFFFF};
    for (int32_t m : kMax)
        if (lo <= m && hi > m) { Utf8Split(lo, m, out); Utf8Split(m + 1, hi, out); return; }
    int n = EncLen(lo);
    for (int i = 1; i < n; i++) {
        int32_t m = (1 << (6 * i)) - 1;
        if ((lo & ~m) != (hi & ~m)) {
            if ((lo & m) != 0) { Utf8Split(lo, lo | m, out); Utf8Split((lo | m) + 1, hi, out); return; }
            if ((hi & m) != m) { Utf8Split(lo, (hi & ~m) - 1, out); Utf8Split(hi & ~m, hi, out); return; }
        }
    }
    uint8_t a[4], b[4];
    Enc(lo, a); Enc(hi, b);
    Seq s;
    for (int k = 0; k < n; k++) s.emplace_back(a[k], b[k]);
    out.push_back(s);
}

class Nfa {
public:
    std::vector<NState> st;
    bool uses_line = false, uses_word = false;
    // rune mode (BuildBitNfa): a class is one K::Rune state matching a decoded
    // rune instead of a UTF-8 byte trie; byte-level ops are not available
    bool rune_mode = false, byte_ops = false;
    std::vector<RuneSet> rsets;

    int New(K k) { st.emplace_back(); st.back().k = k; return (int)st.size() - 1; }
    int Compile(const Node *x, int next);
    int CompileClass(const RuneSet &c, int next);

private:
    std::map<std::pair<std::vector<uint16_t>, int>, int> suffix_;  // shared continuation chains
};

int Nfa::CompileClass(const RuneSet &c, int next) {
    if (rune_mode) {
        int r = New(K::Rune);
        st[r].rset = (int)rsets.size();
        st[r].out = next;
        rsets.push_back(c);
        return r;
    }
    int e = New(K::Byte);
    std::vector<Seq> seqs;
    for (auto &r : c.r) Utf8Split(r.first, r.second, seqs);
    for (auto &sq : seqs) {
        int to = next;
        std::vector<uint16_t> key;
        for (int k = (int)sq.size() - 1; k >= 1; k--) {
            key.push_back((uint16_t)(sq[k].first << 8 | sq[k].second));
            auto it = suffix_.find({key, next});
            if (it != suffix_.end()) { to = it->second; continue; }
            int s = New(K::Byte);
            st[s].tr.push_back({sq[k].first, sq[k].second, G_NONE, to});
            suffix_[{key, next}] = s;
            to = s;
        }
        st[e].tr.push_back({sq[0].first, sq[0].second, G_NONE, to});
    }
    if (c.contains(0xFFFD)) {  // bytes that utf8.DecodeRune reads as RuneError, width 1
        st[e].tr.push_back({0x80, 0xC1, G_NONE, next});
        st[e].tr.push_back({0xF5, 0xFF, G_NONE, next});
        st[e].tr.push_back({0xC2, 0xDF, G2, next});
        st[e].tr.push_back({0xE0, 0xE0, GE0, next});
        st[e].tr.push_back({0xE1, 0xEC, G3, next});
        st[e].tr.push_back({0xED, 0xED, GED, next});
        st[e].tr.push_back({0xEE, 0xEF, G3, next});
        st[e].tr.push_back({0xF0, 0xF0, GF0, next});
        st[e].tr.push_back({0xF1, 0xF3, G4, next});
        st[e].tr.push_back({0xF4, 0xF4, GF4, next});
    }
    return e;
}

int Nfa::Compile(const Node *x, int next) {
    switch (x->op) {
    case Op::NoMatch: return New(K::Byte);
    case Op::Empty: return next;
    case Op::Class: return x->cls.empty() ? New(K::Byte) : CompileClass(x->cls, next);
    case Op::AnyNotNL: { RuneSet s; s.add(0, 9); s.add(11, 0x10FFFF); return CompileClass(s, next); }
    case Op::Any: { RuneSet s; s.add(0, 0x10FFFF); return CompileClass(s, next); }
    case Op::BeginLine: case Op::EndLine: case Op::BeginText: case Op::EndText:
    case Op::WordBoundary: case Op::NoWordBoundary: {
        int s = New(K::Assert);
        uint8_t c = 0;
        switch (x->op) {
        case Op::BeginLine: c = C_BOL; uses_line = true; break;
        case Op::EndLine: c = C_EOL; uses_line = true; break;
        case Op::BeginText: c = C_BOT; break;
        case Op::EndText: c = C_EOT; break;
        case Op::WordBoundary: c = C_WB; uses_word = true; break;
        default: c = C_NWB; uses_word = true; break;
        }
        st[s].cond = c;
        st[s].out = next;
        return s;
    }
    case Op::ByteString: {
        byte_ops |= rune_mode;
        int pc = next;
        for (int i = (int)x->bytes.size() - 1; i >= 0; i--) {
            int s = New(K::Byte);
            uint8_t b = (uint8_t)x->bytes[i];
            st[s].tr.push_back({b, b, G_NONE, pc});
            pc = s;
        }
        return pc;
    }
    case Op::AnyBytes: {  // [\x00-\xff]* over raw bytes
        byte_ops |= rune_mode;
        int s = New(K::Split);
        int b = New(K::Byte);
        st[b].tr.push_back({0x00, 0xFF, G_NONE, s});
        st[s].out = b; st[s].out1 = next;
        return s;
    }
    case Op::Concat: {
        int pc = next;
        for (int i = (int)x->sub.size() - 1; i >= 0; i--) pc = Compile(x->sub[i].get(), pc);
        return pc;
    }
    case Op::Alternate: {
        int pc = Compile(x->sub.back().get(), next);
        for (int i = (int)x->sub.size() - 2; i >= 0; i--) {
            int a = Compile(x->sub[i].get(), next);
            int s = New(K::Split);
            st[s].out = a; st[s].out1 = pc;
            pc = s;
        }
        return pc;
    }
    case Op::Star: {
        int s = New(K::Split);
        int body = Compile(x->sub[0].get(), s);
        st[s].out = body; st[s].out1 = next;
        return s;
    }
    case Op::Plus: {
        int s = New(K::Split);
        int body = Compile(x->sub[0].get(), s);
        st[s].out = body; st[s].out1 = next;
        return body;
    }
    case Op::Quest: {
        int body = Compile(x->sub[0].get(), next);
        int s = New(K::Split);
        st[s].out = body; st[s].out1 = next;
        return s;
    }
    case Op::Repeat: {
        int pc = next;
        if (x->max < 0) {
            int s = New(K::Split);
            int body = Compile(x->sub[0].get(), s);
            st[s].out = body; st[s].out1 = next;
            pc = s;
        } else {
            for (int k = x->min; k < x->max; k++) {
                int body = Compile(x->sub[0].get(), pc);
                int s = New(K::Split);
                st[s].out = body; st[s].out1 = next;
                pc = s;
            }
        }
        for (int k = 0; k < x->min; k++) pc = Compile(x->sub[0].get(), pc);
        return pc;
    }
    default: break;
    }
    return New(K::Byte);
}

struct VecHash {
    size_t operator()(const std::vector<int> &v) const {
        size_t h = 1469598103934665603ull;
        for (int x : v) { h ^= (size_t)x; h *= 1099511628211ull; }
        return h;
    }
};

}  // namespace

bool DFA::absorbing(int s) const {
    for (int c = 0; c < ncls; c++) if (next[(size_t)s * ncls + c] != s) return false;
    return true;
}

bool BuildDFA(const std::vector<Pattern> &pats, int max_states, DFA *out, std::string *err) {
    Nfa nfa;
    const int np = (int)pats.size();
    const int words = (np + 63) / 64;
    std::vector<int> entries(np);
    bool any_unanchored = false;
    for (int k = 0; k < np; k++) {
        int m = nfa.New(K::Match);
        nfa.st[m].acc = k;
        if (!pats[k].anchored) {
            any_unanchored = true;
            int d = nfa.New(K::Byte);
            nfa.st[d].acc = k;
            nfa.st[d].tr.push_back({0x00, 0xFF, G_NONE, d});
            nfa.st[m].done = d;
        }
        entries[k] = nfa.Compile(pats[k].ast, m);
    }
    std::vector<int> start;
    for (int k = 0; k < np; k++) if (pats[k].anchored) start.push_back(entries[k] * 8);
    if (any_unanchored) {
        // search loop over whole runes (Go starts a match only at rune boundaries)
        int s0 = nfa.New(K::Split);
        RuneSet any; any.add(0, 0x10FFFF);
        int loop = nfa.CompileClass(any, s0);
        int fan = -1;
        for (int k = np - 1; k >= 0; k--) {
            if (pats[k].anchored) continue;
            if (fan < 0) { fan = entries[k]; continue; }
            int s = nfa.New(K::Split);
            nfa.st[s].out = entries[k]; nfa.st[s].out1 = fan;
            fan = s;
        }
        nfa.st[s0].out = loop; nfa.st[s0].out1 = fan;
        start.push_back(s0 * 8);
    }
    std::sort(start.begin(), start.end());
    start.erase(std::unique(start.begin(), start.end()), start.end());

    // ---- byte intervals for the construction
    bool cut[257] = {false};
    cut[0] = cut[256] = true;
    for (auto &s : nfa.st)
        for (auto &t : s.tr) { cut[t.lo] = true; cut[t.hi + 1] = true; }
    for (int g = 1; g < 8; g++) { cut[kGuard[g].lo] = true; cut[kGuard[g].hi + 1] = true; }
    if (nfa.uses_line) { cut['\n'] = cut['\n' + 1] = true; }
    if (nfa.uses_word) for (int b = 0; b < 256; b++) if (IsWordByte(b) != IsWordByte(b - 1)) cut[b] = true;
    std::vector<int> ilo;
    for (int b = 0; b < 256; b++) if (cut[b]) ilo.push_back(b);
    const int nint = (int)ilo.size();
    uint8_t int_of[256];
    for (int i = 0; i < nint; i++) {
        int hi = i + 1 < nint ? ilo[i + 1] : 256;
        for (int b = ilo[i]; b < hi; b++) int_of[b] = (uint8_t)i;
    }
    const uint8_t ctx_mask = P_START | (nfa.uses_line ? P_NL : 0) | (nfa.uses_word ? P_WORD : 0);

    // closure under empty-width condition `cond`
    std::vector<int> mark(nfa.st.size() * 8, -1);
    int epoch = 0;
    std::vector<int> stack;
    auto closure = [&](const std::vector<int> &th, uint8_t cond, std::vector<int> &byte_th, std::vector<uint64_t> *acc) {
        epoch++;
        byte_th.clear();
        stack.assign(th.rbegin(), th.rend());
        while (!stack.empty()) {
            int t = stack.back(); stack.pop_back();
            if (mark[t] == epoch) continue;
            mark[t] = epoch;
            int q = t >> 3, g = t & 7;
            const NState &s = nfa.st[q];
            switch (s.k) {
            case K::Split: stack.push_back(s.out1 * 8 + g); stack.push_back(s.out * 8 + g); break;
            case K::Assert: if ((s.cond & cond) == s.cond) stack.push_back(s.out * 8 + g); break;
            case K::Match:
                if (acc) (*acc)[s.acc >> 6] |= 1ull << (s.acc & 63);
                if (s.done >= 0) stack.push_back(s.done * 8 + g);
                break;
            case K::Byte:
                if (acc && s.acc >= 0) (*acc)[s.acc >> 6] |= 1ull << (s.acc & 63);
                if (!s.tr.empty()) byte_th.push_back(t);
                break;
            }
        }
    };
    auto cond_for = [&](uint8_t prev, int b) -> uint8_t {
        uint8_t c = 0;
        if (prev & P_START) c |= C_BOT | C_BOL;
        if (prev & P_NL) c |= C_BOL;
        bool pw = (prev & P_WORD) != 0;
        if (b < 0) { c |= C_EOT | C_EOL; c |= pw ? C_WB : C_NWB; }
        else { if (b == '\n') c |= C_EOL; c |= (pw != IsWordByte(b)) ? C_WB : C_NWB; }
        return c;
    };

    struct Key { std::vector<int> th; uint8_t ctx; };
    struct KeyHash {
        size_t operator()(const Key &k) const { return VecHash()(k.th) * 31 + k.ctx; }
    };
    struct KeyEq {
        bool operator()(const Key &a, const Key &b) const { return a.ctx == b.ctx && a.th == b.th; }
    };
    std::unordered_map<Key, int, KeyHash, KeyEq> index;
    std::vector<Key> keys;
    keys.push_back({{}, 0});  // dead state 0
    std::vector<std::vector<int>> trans;  // per state per interval
    std::vector<std::vector<uint64_t>> accept;
    auto intern = [&](Key &&k) -> int {
        if (k.th.empty()) return 0;
        auto it = index.find(k);
        if (it != index.end()) return it->second;
        int id = (int)keys.size();
        index.emplace(k, id);
        keys.push_back(std::move(k));
        return id;
    };
    int s_start = intern(Key{start, (uint8_t)(P_START & ctx_mask)});
    std::vector<int> bth, nxt;
    for (size_t cur = 0; cur < keys.size(); cur++) {
        if ((int)keys.size() > max_states) {
            if (err) *err = "DFA state budget exceeded";
            return false;
        }
        trans.emplace_back(nint, 0);
        accept.emplace_back(words, 0);
        if (cur == 0) continue;
        const Key key = keys[cur];
        closure(key.th, cond_for(key.ctx, -1), bth, &accept[cur]);
        uint8_t last_cond = 0xFF;
        std::vector<int> cl;
        for (int iv = 0; iv < nint; iv++) {
            int b = ilo[iv];
            uint8_t c = cond_for(key.ctx, b);
            if (c != last_cond) { closure(key.th, c, cl, nullptr); last_cond = c; }
            nxt.clear();
            for (int t : cl) {
                uint8_t g2 = GuardStep((uint8_t)(t & 7), (uint8_t)b);
                if (g2 == G_DIE) continue;
                for (const BTr &tr : nfa.st[t >> 3].tr)
                    if (b >= tr.lo && b <= tr.hi) nxt.push_back(tr.to * 8 + (g2 != G_NONE ? g2 : tr.guard));
            }
            std::sort(nxt.begin(), nxt.end());
            nxt.erase(std::unique(nxt.begin(), nxt.end()), nxt.end());
            uint8_t pc = 0;
            if (b == '\n') pc |= P_NL;
            if (IsWordByte(b)) pc |= P_WORD;
            trans[cur][iv] = intern(Key{nxt, (uint8_t)(pc & ctx_mask)});
        }
    }
    int n = (int)keys.size();
    if (n > max_states) {
        if (err) *err = "DFA state budget exceeded";
        return false;
    }

    // ---- Moore minimisation; state 0 (dead) keeps its own block id 0
    std::vector<int> blk(n);
    {
        std::map<std::vector<uint64_t>, int> sig;
        sig[std::vector<uint64_t>(words, 0)] = 0;  // never accepts, as dead
        for (int s = 0; s < n; s++) {
            auto it = sig.find(accept[s]);
            if (it == sig.end()) it = sig.emplace(accept[s], (int)sig.size()).first;
            blk[s] = it->second;
        }
    }
    int nb = 0;
    for (;;) {
        std::map<std::vector<int>, int> sig;
        std::vector<int> nblk(n);
        // the block holding the dead state must stay id 0
        std::vector<int> v0; v0.push_back(blk[0]);
        for (int iv = 0; iv < nint; iv++) v0.push_back(blk[trans[0][iv]]);
        sig[v0] = 0;
        for (int s = 0; s < n; s++) {
            std::vector<int> v; v.reserve(nint + 1);
            v.push_back(blk[s]);
            for (int iv = 0; iv < nint; iv++) v.push_back(blk[trans[s][iv]]);
            auto it = sig.find(v);
            if (it == sig.end()) it = sig.emplace(v, (int)sig.size()).first;
            nblk[s] = it->second;
        }
        int cnt = (int)sig.size();
        bool stable = cnt == nb;
        blk.swap(nblk);
        nb = cnt;
        if (stable) break;
    }
    // ---- byte classes: intervals with identical transition columns
    std::map<std::vector<int>, int> colmap;
    std::vector<int> icls(nint);
    std::vector<int> rep;  // interval representative per class
    for (int iv = 0; iv < nint; iv++) {
        std::vector<int> col(nb, -1);
        for (int s = 0; s < n; s++) col[blk[s]] = blk[trans[s][iv]];
        auto it = colmap.find(col);
        if (it == colmap.end()) { it = colmap.emplace(col, (int)rep.size()).first; rep.push_back(iv); }
        icls[iv] = it->second;
    }
    out->nstates = nb;
    out->ncls = (int)rep.size();
    out->npatterns = np;
    out->start = blk[s_start];
    for (int b = 0; b < 256; b++) out->cls[b] = (uint8_t)icls[int_of[b]];
    out->next.assign((size_t)nb * out->ncls, 0);
    out->accept.assign(nb, std::vector<uint64_t>(words, 0));
    for (int s = 0; s < n; s++) {
        out->accept[blk[s]] = accept[s];
        for (int c = 0; c < out->ncls; c++) out->next[(size_t)blk[s] * out->ncls + c] = (uint16_t)blk[trans[s][rep[c]]];
    }
    if (nb > 65535) { if (err) *err = "DFA too large"; return false; }
    return true;
}

bool BuildBitNfa(const Pattern &p, int max_positions, BitNfa *out, std::string *err, int dense_words) {
    Nfa nfa;
    nfa.rune_mode = true;
    RuneSet any;
    any.add(0, 0x10FFFF);
    const int mt = nfa.New(K::Match);
    nfa.st[mt].acc = 0;
    if (!p.anchored) {  // Go regexp.Match: a sticky "done" state after the first match
        int d = nfa.CompileClass(any, -1);
        nfa.st[d].out = d;
        nfa.st[d].acc = 0;
        nfa.st[mt].done = d;
    }
    const int entry = nfa.Compile(p.ast, mt);
    if (nfa.byte_ops) {
        if (err) *err = "byte-level matcher in the NFA fallback";
        return false;
    }
    int start = entry;
    if (!p.anchored) {  // search loop over whole runes, as in BuildDFA
        int s0 = nfa.New(K::Split);
        int loop = nfa.CompileClass(any, s0);
        nfa.st[s0].out = loop;
        nfa.st[s0].out1 = entry;
        start = s0;
    }
    // ---- positions: the rune states; 0 = virtual start
    const int ns = (int)nfa.st.size();
    std::vector<int> pos_of(ns, -1), to_of{start}, rset_of{-1};
    for (int q = 0; q < ns; q++)
        if (nfa.st[q].k == K::Rune) {
            pos_of[q] = (int)to_of.size();
            to_of.push_back(nfa.st[q].out);
            rset_of.push_back(nfa.st[q].rset);
        }
    const int m = (int)to_of.size();
    if (m > max_positions) {
        if (err) *err = "regex needs " + std::to_string(m) + " NFA positions (limit " + std::to_string(max_positions) + ")";
        return false;
    }
    const int W = (m + 63) / 64;
    // ---- empty-width condition classes: the achievable conditions reduced
    // to the bits some assertion of the pattern tests
    uint8_t relevant = 0;
    for (auto &st : nfa.st)
        if (st.k == K::Assert) relevant |= st.cond;
    auto cond_for = [](uint8_t prev, int b) -> uint8_t {  // as in BuildDFA
        uint8_t c = 0;
        if (prev & P_START) c |= C_BOT | C_BOL;
        if (prev & P_NL) c |= C_BOL;
        bool pw = (prev & P_WORD) != 0;
        if (b < 0) { c |= C_EOT | C_EOL; c |= pw ? C_WB : C_NWB; }
        else { if (b == '\n') c |= C_EOL; c |= (pw != IsWordByte(b)) ? C_WB : C_NWB; }
        return c;
    };
    std::vector<uint8_t> cls_cond;  // class -> reduced condition
    memset(out->condmap, 0, sizeof out->condmap);
    for (uint8_t prev : {(uint8_t)P_START, (uint8_t)0, (uint8_t)P_NL, (uint8_t)P_WORD})
        for (int b : {-1, (int)'\n', (int)'a', (int)' '}) {
            const uint8_t raw = cond_for(prev, b), red = raw & relevant;
            int k = (int)(std::find(cls_cond.begin(), cls_cond.end(), red) - cls_cond.begin());
            if (k == (int)cls_cond.size()) cls_cond.push_back(red);
            out->condmap[raw & 63] = (uint8_t)k;
        }
    const int K = (int)cls_cond.size();
    // ---- follow sets and acceptance per class (epsilon closure of each target)
    out->m = m;
    out->W = W;
    out->K = K;
    out->sparse = W > dense_words;
    if (out->sparse) {
        out->row_of.assign((size_t)K * m, 0);
        out->row_ptr.assign(1, 0);
    } else {
        out->follow.assign((size_t)K * m * W, 0);
    }
    out->acc.assign((size_t)K * W, 0);
    std::vector<int> mark(ns, -1), stack;
    std::vector<uint64_t> tmp(out->sparse ? W : 0);  // a sparse row being built
    std::vector<uint32_t> touched;
    int epoch = 0;
    for (int k = 0; k < K; k++) {
        const uint8_t cond = cls_cond[k];
        std::vector<int> memo_to(ns, -1);  // target state -> position whose row is already computed
        for (int pp = 0; pp < m; pp++) {
            const int to = to_of[pp];
            if (memo_to[to] >= 0) {
                const int src = memo_to[to];
                if (out->sparse) {
                    out->row_of[(size_t)k * m + pp] = out->row_of[(size_t)k * m + src];
                } else {
                    const uint64_t *sr = &out->follow[((size_t)k * m + src) * W];
                    std::copy(sr, sr + W, &out->follow[((size_t)k * m + pp) * W]);
                }
                if ((out->acc[(size_t)k * W + src / 64] >> (src % 64)) & 1)
                    out->acc[(size_t)k * W + pp / 64] |= 1ull << (pp % 64);
                continue;
            }
            memo_to[to] = pp;
            uint64_t *row = out->sparse ? tmp.data() : &out->follow[((size_t)k * m + pp) * W];
            epoch++;
            bool accepts = false;
            stack.assign(1, to);
            while (!stack.empty()) {
                int q = stack.back(); stack.pop_back();
                if (mark[q] == epoch) continue;
                mark[q] = epoch;
                const NState &st = nfa.st[q];
                switch (st.k) {
                case K::Split: stack.push_back(st.out1); stack.push_back(st.out); break;
                case K::Assert: if ((st.cond & cond) == st.cond) stack.push_back(st.out); break;
                case K::Match: accepts = true; if (st.done >= 0) stack.push_back(st.done); break;
                case K::Rune: {
                    if (st.acc >= 0) accepts = true;
                    const int e = pos_of[q];
                    if (out->sparse && !row[e / 64]) touched.push_back((uint32_t)(e / 64));
                    row[e / 64] |= 1ull << (e % 64);
                    break;
                }
                case K::Byte: break;  // an empty class: matches nothing
                }
            }
            if (accepts) out->acc[(size_t)k * W + pp / 64] |= 1ull << (pp % 64);
            if (out->sparse) {  // the row's non-zero words, in word order
                std::sort(touched.begin(), touched.end());
                out->row_of[(size_t)k * m + pp] = (uint32_t)(out->row_ptr.size() - 1);
                for (uint32_t w : touched) {
                    out->pair_w.push_back(w);
                    out->pair_m.push_back(row[w]);
                    row[w] = 0;
                }
                touched.clear();
                out->row_ptr.push_back((uint32_t)out->pair_w.size());
                if (out->pair_w.size() > (1u << 27)) {
                    if (err) *err = "NFA follow tables exceed 2^27 entries";
                    return false;
                }
            }
        }
    }
    // ---- rune intervals on which every position's class is constant
    std::vector<int32_t> cuts{0, 0x110000};
    for (auto &rs : nfa.rsets)
        for (auto &r : rs.r) { cuts.push_back(r.first); cuts.push_back(r.second + 1); }
    std::sort(cuts.begin(), cuts.end());
    cuts.erase(std::unique(cuts.begin(), cuts.end()), cuts.end());
    cuts.pop_back();  // 0x110000 closes the last interval
    out->ivl_lo.assign(cuts.begin(), cuts.end());
    const size_t niv = cuts.size();
    out->b.assign(niv * W, 0);
    for (int pp = 1; pp < m; pp++)
        for (auto &r : nfa.rsets[rset_of[pp]].r)
            for (size_t iv = std::lower_bound(cuts.begin(), cuts.end(), r.first) - cuts.begin();
                 iv < niv && cuts[iv] <= r.second; iv++)
                out->b[iv * W + pp / 64] |= 1ull << (pp % 64);
    return true;
}

std::vector<uint64_t> RunDFA(const DFA &d, const uint8_t *s, size_t n) {
    int st = d.start;
    for (size_t i = 0; i < n && st != 0; i++) st = d.next[(size_t)st * d.ncls + d.cls[s[i]]];
    return d.accept[st];
}

}  // namespace re
}  // namespace l7
