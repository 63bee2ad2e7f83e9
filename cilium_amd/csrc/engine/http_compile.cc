#include "http_compile.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>

#include "../regex/re_dfa.h"
#include "nfa_pool.h"

namespace l7 {

namespace {

// Header lookup as the filter sees it: pseudo headers from the request line /
// Host; "host" and x-envoy-original-dst-host are never visible as regular
// headers (the codec maps Host to :authority; cilium_l7policy.cc:128 strips
// the other); unknown pseudo headers are never present.
constexpr int kSlotNever = 0xFF;
int FixedSlot(const std::string &name) {
    if (name == ":method") return SLOT_METHOD;
    if (name == ":path") return SLOT_PATH;
    if (name == ":authority") return SLOT_AUTHORITY;
    if (name == "host" || name == "x-envoy-original-dst-host") return kSlotNever;
    if (!name.empty() && name[0] == ':') return kSlotNever;
    return -1;
}

struct Pat {
    HM type;
    std::string value;
    bool invert;
    std::shared_ptr<re::Node> ast;
};

std::unique_ptr<re::Node> MakeBytes(const std::string &v) {
    auto n = std::make_unique<re::Node>(re::Op::ByteString);
    n->bytes = v;
    return n;
}

std::unique_ptr<re::Node> PatternAst(const Pat &p, std::string *err) {
    using re::Node;
    using re::Op;
    switch (p.type) {
    case HM::Exact:
        if (p.value.empty()) return std::make_unique<Node>(Op::AnyBytes);
        return MakeBytes(p.value);
    case HM::Present: return std::make_unique<Node>(Op::AnyBytes);
    case HM::Prefix: {
        auto c = std::make_unique<Node>(Op::Concat);
        c->sub.push_back(MakeBytes(p.value));
        c->sub.push_back(std::make_unique<Node>(Op::AnyBytes));
        return c;
    }
    case HM::Suffix: {
        auto c = std::make_unique<Node>(Op::Concat);
        c->sub.push_back(std::make_unique<Node>(Op::AnyBytes));
        c->sub.push_back(MakeBytes(p.value));
        return c;
    }
    case HM::Regex: return nullptr;  // uses p.ast directly
    case HM::Range: break;
    }
    *err = "range_match header matchers are not supported by the device compiler";
    return nullptr;
}

}  // namespace

int HttpCompiler::RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, bool proxylib,
                             std::string *err) {
    std::vector<const HttpRule *> items;
    uint8_t terminal = V_DENY;
    if (proxylib && policy >= 0 && policy < (int)ps_->policies.size()) {
        // proxylib "http" parser: PortNetworkPolicies.Matches (policymap.go:208-236)
        // -- exact port then port 0, entries proxylib installs only, no entry => drop
        const PortPolicy *ex, *wc;
        ps_->policies[policy].Lookup(ingress, port, &ex, &wc);
        bool decided = false;
        for (const PortPolicy *pp : {ex, wc}) {
            if (!pp || !pp->px_installed) continue;
            if (!pp->px_have_l7 || pp->rules.empty()) { terminal = V_ALLOW; decided = true; break; }  // :173-186
            for (auto &r : pp->rules) {
                if (!r.RemoteOk(remote)) continue;
                if (r.NumL7() == 0) { terminal = V_ALLOW; decided = true; break; }  // empty L7 set (:106-108)
                if (r.type == PortRule::Http)
                    for (auto &h : r.http) items.push_back(&h);
            }
            if (decided) break;
        }
    } else if (!proxylib && policy >= 0 && policy < (int)ps_->policies.size()) {
        const NetworkPolicy &np = ps_->policies[policy];
        const PortPolicy *ex, *wc;
        np.Lookup(ingress, port, &ex, &wc);
        bool decided = false;
        for (const PortPolicy *pp : {ex, wc}) {
            if (!pp) continue;
            if (!pp->has_http || pp->rules.empty()) { terminal = V_ALLOW; decided = true; break; }
            for (auto &r : pp->rules) {
                if (!r.RemoteOk(remote)) continue;
                if (r.type == PortRule::Http && !r.http.empty()) {
                    for (auto &h : r.http) items.push_back(&h);
                } else {  // no HTTP rules in this group: any payload from this remote
                    terminal = V_ALLOW;
                    decided = true;
                    break;
                }
            }
            if (decided) break;
        }
        if (!decided) terminal = (ex || wc) ? V_DENY : V_ALLOW;
    }
    std::vector<int> ids;
    for (auto *h : items) ids.push_back(h->id);
    auto key = std::make_pair(ids, (int)terminal);
    auto it = cache_.find(key);
    if (it != cache_.end()) return it->second;
    int rs = Compile(items, terminal, err);
    if (rs >= 0) cache_.emplace(key, rs);
    return rs;
}

namespace {

bool IsTchar(uint8_t c) {
    if ((c >= '0' && c <= '9') || (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z')) return true;
    return c && strchr("!#$%&'*+-.^_`|~", c) != nullptr;
}

// Trie automaton over lower-cased header-name bytes (device_tables.h, NI_*).
struct NameDfa {
    uint8_t cls[256] = {0};
    int ncls = 2;
    std::vector<uint16_t> trans;  // [state][class]
    std::vector<uint8_t> info;    // [state]
};

// The names the framer must recognise, with their NI_* flags (a custom name
// equal to a fixed one merges into it).
std::vector<std::pair<std::string, uint8_t>> NameCandidates(const std::vector<std::string> &custom) {
    std::vector<std::pair<std::string, uint8_t>> cands = {
        {"host", NI_HOST}, {"content-length", NI_CL}, {"transfer-encoding", NI_TE}};
    for (size_t q = 0; q < custom.size(); q++) {
        bool merged = false;
        for (auto &c : cands)
            if (c.first == custom[q]) { c.second |= (uint8_t)(q + 1); merged = true; }
        if (!merged) cands.emplace_back(custom[q], (uint8_t)(q + 1));
    }
    return cands;
}

// DevNameEnt table of the candidates that a <= 15-byte [0-9A-Za-z-] name can
// equal (device_tables.h); bits = 0 if no collision-free multiplier is found.
std::vector<DevNameEnt> BuildNameTable(const std::vector<std::string> &custom, uint32_t *bits_out, uint32_t *mul_out) {
    std::vector<DevNameEnt> ents;
    for (auto &cd : NameCandidates(custom)) {
        const std::string &s = cd.first;
        bool ok = !s.empty() && s.size() <= 15;
        for (unsigned char ch : s) ok = ok && ((ch >= '0' && ch <= '9') || (ch >= 'a' && ch <= 'z') || ch == '-');
        if (!ok) continue;  // no fast-path name can equal it
        DevNameEnt e{};
        memcpy(e.w, s.data(), s.size());
        e.len = (uint8_t)s.size();
        e.info = cd.second;
        ents.push_back(e);
    }
    uint32_t bits = 1;
    while ((1u << bits) < 2 * ents.size()) bits++;
    uint64_t seed = 0x9E3779B97F4A7C15ull;
    for (; bits <= 8; bits++) {
        for (int tries = 0; tries < 4096; tries++) {
            seed = seed * 6364136223846793005ull + 1442695040888963407ull;
            const uint32_t mul = (uint32_t)(seed >> 32) | 1u;
            std::vector<DevNameEnt> tab((size_t)1 << bits);
            bool clash = false;
            for (auto &e : ents) {
                DevNameEnt &t = tab[l7_name_hash(e.w[0], e.w[1], e.w[2], e.w[3], e.len, mul, bits)];
                if (t.len) { clash = true; break; }
                t = e;
            }
            if (!clash) {
                *bits_out = bits;
                *mul_out = mul;
                return tab;
            }
        }
    }
    *bits_out = 0;
    *mul_out = 0;
    return {};
}

NameDfa BuildNameDfa(const std::vector<std::string> &custom) {
    const std::vector<std::pair<std::string, uint8_t>> cands = NameCandidates(custom);
    NameDfa d;
    // classes: 0 = not a tchar, 1 = tchar spelling none of the names, 2.. = name bytes
    int byte_cls[256];
    for (int c = 0; c < 256; c++) byte_cls[c] = -1;
    for (auto &cd : cands) {
        bool ok = !cd.first.empty();
        for (unsigned char ch : cd.first) ok = ok && IsTchar(ch) && !(ch >= 'A' && ch <= 'Z');
        if (!ok) continue;  // a name no valid header line can carry: never present
        for (unsigned char ch : cd.first)
            if (byte_cls[ch] < 0) byte_cls[ch] = d.ncls++;
    }
    for (int c = 0; c < 256; c++) {
        if (!IsTchar((uint8_t)c)) { d.cls[c] = 0; continue; }
        int lc = (c >= 'A' && c <= 'Z') ? c + 32 : c;
        d.cls[c] = (uint8_t)(byte_cls[lc] >= 0 ? byte_cls[lc] : 1);
    }
    // trie: 0 bad, 1 other, 2 root
    std::vector<std::map<int, int>> kids(3);
    std::vector<uint8_t> info(3, 0);
    for (auto &cd : cands) {
        bool ok = !cd.first.empty();
        for (unsigned char ch : cd.first) ok = ok && IsTchar(ch) && !(ch >= 'A' && ch <= 'Z');
        if (!ok) continue;
        int s = kNameStart;
        for (unsigned char ch : cd.first) {
            int k = d.cls[ch];
            auto it = kids[s].find(k);
            if (it == kids[s].end()) {
                kids.emplace_back();
                info.push_back(0);
                int ns = (int)kids.size() - 1;
                kids[s][k] = ns;
                s = ns;
            } else {
                s = it->second;
            }
        }
        info[s] |= cd.second;
    }
    const int ns = (int)kids.size();
    d.trans.assign((size_t)ns * d.ncls, kNameOther);
    for (int s = 0; s < ns; s++)
        for (int k = 0; k < d.ncls; k++) {
            uint16_t to = kNameOther;
            if (s == kNameBad || k == 0) to = kNameBad;
            else if (s != kNameOther) {
                auto it = kids[s].find(k);
                if (it != kids[s].end()) to = (uint16_t)it->second;
            }
            d.trans[(size_t)s * d.ncls + k] = to;
        }
    d.info = info;
    return d;
}

// Renumber d's states so that those absorbing on header-token bytes (HT, SP,
// VCHAR, obs-text: each such byte leads back to the state) come last,
// [absorb, nstates); the dead state keeps number 0.  The kernel stops walking
// a token once its state is absorbing: the rest of the token cannot change it.
uint32_t SortAbsorbing(re::DFA &d) {
    const int n = d.nstates;
    std::vector<char> ab(n, 0);
    for (int s = 1; s < n; s++) {
        bool a = true;
        for (int b = 0; b < 256 && a; b++) {
            const bool token_byte = b == '\t' || (b >= 0x20 && b != 0x7F);
            if (token_byte && d.next[(size_t)s * d.ncls + d.cls[b]] != s) a = false;
        }
        ab[s] = a;
    }
    std::vector<int> order{0};
    for (int s = 1; s < n; s++)
        if (!ab[s]) order.push_back(s);
    const uint32_t absorb = (uint32_t)order.size();
    for (int s = 1; s < n; s++)
        if (ab[s]) order.push_back(s);
    std::vector<int> id(n);
    for (int i = 0; i < n; i++) id[order[i]] = i;
    std::vector<uint16_t> next((size_t)n * d.ncls);
    std::vector<std::vector<uint64_t>> acc(n);
    for (int i = 0; i < n; i++) {
        for (int c = 0; c < d.ncls; c++)
            next[(size_t)i * d.ncls + c] = (uint16_t)id[d.next[(size_t)order[i] * d.ncls + c]];
        acc[i] = d.accept[order[i]];
    }
    d.next.swap(next);
    d.accept.swap(acc);
    d.start = id[d.start];
    return absorb;
}

template <class T>
uint32_t Append(std::vector<uint8_t> &img, const T *p, size_t n) {
    size_t off = (img.size() + 15) & ~(size_t)15;
    img.resize(off + n * sizeof(T));
    if (n) memcpy(img.data() + off, p, n * sizeof(T));
    return (uint32_t)off;
}

}  // namespace

int HttpCompiler::Compile(const std::vector<const HttpRule *> &rules, uint8_t terminal, std::string *err) {
    compiled++;
    // custom header names used anywhere in the rule set
    std::vector<std::string> custom;
    for (auto *r : rules)
        for (auto &m : r->m)
            if (FixedSlot(m.name) < 0 && std::find(custom.begin(), custom.end(), m.name) == custom.end()) custom.push_back(m.name);
    if ((int)custom.size() > kMaxCustomHeaders) {
        *err = "rule set references more than 8 distinct custom headers";
        return -1;
    }
    auto slot_of = [&](const std::string &name) {
        int s = FixedSlot(name);
        if (s >= 0) return s;
        return SLOT_CUSTOM0 + (int)(std::find(custom.begin(), custom.end(), name) - custom.begin());
    };
    const size_t nr = rules.size();
    const size_t nchunks = (nr + 63) / 64;
    if (nchunks > 255) { *err = "rule set has more than 16320 HTTP rules"; return -1; }
    auto bit = [](size_t r) { return 1ull << (r & 63); };
    std::vector<uint64_t> all(nchunks, 0), init(nchunks, 0);
    for (size_t r = 0; r < nr; r++) all[r >> 6] |= bit(r);
    init = all;
    // absent[s][c]: rules of chunk c not constrained on slot s.  A matcher on
    // a missing header never holds (HeaderUtility::matchHeaders returns false
    // before invert_match applies), so constrained rules drop out.
    std::vector<uint64_t> absent((size_t)kNumSlots * nchunks);
    for (int s = 0; s < kNumSlots; s++)
        for (size_t c = 0; c < nchunks; c++) absent[s * nchunks + c] = all[c];
    // matchers per slot: (rule index, matcher)
    std::map<int, std::vector<std::pair<size_t, const HeaderMatcher *>>> by_slot;
    for (size_t r = 0; r < nr; r++)
        for (auto &m : rules[r]->m) {
            int s = slot_of(m.name);
            if (s == kSlotNever) { init[r >> 6] &= ~bit(r); continue; }
            by_slot[s].emplace_back(r, &m);
            absent[s * nchunks + (r >> 6)] &= ~bit(r);
        }

    ImgHeader H{};
    H.nchunks = (uint8_t)nchunks;
    H.nhdr = (uint8_t)custom.size();
    H.terminal = terminal;
    struct Built { int slot; re::DFA d; std::vector<uint64_t> masks; uint32_t absorb; };
    std::vector<Built> built;
    struct NfaRef { int slot; uint64_t nfa; int pat; std::vector<uint64_t> masks; };
    std::vector<NfaRef> nfas;
    for (auto &kv : by_slot) {
        const int slot = kv.first;
        H.ref_slots |= (uint16_t)(1u << slot);
        // distinct patterns of this slot
        std::vector<Pat> pats;
        std::vector<std::pair<size_t, int>> rm_pat;  // (rule, pattern)
        for (auto &rm : kv.second) {
            const HeaderMatcher *m = rm.second;
            int idx = -1;
            for (size_t p = 0; p < pats.size(); p++)
                if (pats[p].type == m->type && pats[p].value == m->value && pats[p].invert == m->invert) { idx = (int)p; break; }
            if (idx < 0) { idx = (int)pats.size(); pats.push_back({m->type, m->value, m->invert, m->ast}); }
            rm_pat.emplace_back(rm.first, idx);
        }
        std::vector<std::unique_ptr<re::Node>> owned;
        std::vector<const re::Node *> asts;
        for (auto &p : pats) {
            if (p.type == HM::Regex) { asts.push_back(p.ast.get()); continue; }
            auto a = PatternAst(p, err);
            if (!a) return -1;
            asts.push_back(a.get());
            owned.push_back(std::move(a));
        }
        // build DFAs, halving the pattern set until each fits the budget; a
        // pattern over the budget on its own goes to the NFA fallback
        std::vector<std::vector<int>> groups;
        std::vector<re::DFA> dfas;
        std::vector<int> nfa_pats;
        std::function<bool(std::vector<int>)> build = [&](std::vector<int> sub) -> bool {
            std::vector<re::Pattern> ps;
            for (int p : sub) ps.push_back({asts[p], true});
            re::DFA d;
            std::string e;
            if (re::BuildDFA(ps, max_dfa_states, &d, &e)) { groups.push_back(sub); dfas.push_back(std::move(d)); return true; }
            if (sub.size() == 1) { nfa_pats.push_back(sub[0]); return true; }
            std::vector<int> a(sub.begin(), sub.begin() + sub.size() / 2), b(sub.begin() + sub.size() / 2, sub.end());
            return build(a) && build(b);
        };
        std::vector<int> allp;
        for (size_t p = 0; p < pats.size(); p++) allp.push_back((int)p);
        if (!build(allp)) return -1;
        for (int p : nfa_pats) {
            std::string e;
            auto it = nfa_cache_.find(pats[p].value);
            if (it == nfa_cache_.end()) {
                re::BitNfa n;
                if (re::BuildBitNfa({asts[p], true}, kNfaMaxWords * 64, &n, &e)) {
                    const uint64_t off = AppendDevNfa(n, &img_.nfa_pool, err);
                    if (off == ~0ull) return -1;
                    it = nfa_cache_.emplace(pats[p].value, off).first;
                    img_.nfas++;
                }
            }
            if (it != nfa_cache_.end()) {
                nfas.push_back({slot, it->second, p, {}});
                continue;
            }
            // too many positions for the register NFA: one large DFA if it fits,
            // else the large NFA (sparse rows, state sets in scratch)
            re::DFA d;
            std::string e2, e3;
            re::BitNfa n;
            const bool big = re::BuildBitNfa({asts[p], true}, kNfaMaxPositions, &n, &e3, kNfaMaxWords);
            if (!re::BuildDFA({{asts[p], true}}, big ? LargeNfaDfaBudget(n.m, max_single_dfa_states) : max_single_dfa_states,
                              &d, &e2)) {
                if (!big) {
                    *err = "regex too complex for the device (" + e3 + "): " + pats[p].value;
                    return -1;
                }
                const uint64_t off = AppendDevNfa(n, &img_.nfa_pool, err);
                if (off == ~0ull) return -1;
                it = nfa_cache_.emplace(pats[p].value, off).first;
                img_.nfas++;
                nfas.push_back({slot, it->second, p, {}});
                continue;
            }
            groups.push_back({p});
            dfas.push_back(std::move(d));
        }
        // mask rows of the NFA matchers: [rejected, accepted] x chunks
        for (auto &nf : nfas) {
            if (nf.slot != slot || !nf.masks.empty()) continue;
            nf.masks.resize(2 * nchunks);
            for (int a = 0; a < 2; a++) {
                uint64_t *m = &nf.masks[a * nchunks];
                for (size_t c = 0; c < nchunks; c++) m[c] = all[c];
                for (auto &rp : rm_pat)
                    if (rp.second == nf.pat && (a == 1) == pats[rp.second].invert) m[rp.first >> 6] &= ~bit(rp.first);
            }
        }
        H.max_slot_dfas = (uint8_t)std::max<size_t>(H.max_slot_dfas, dfas.size());
        for (size_t g = 0; g < dfas.size(); g++) {
            Built b{slot, std::move(dfas[g]), {}, 0};
            b.absorb = SortAbsorbing(b.d);  // before the masks, which follow the new numbering
            const std::vector<int> &sub = groups[g];
            std::vector<int> local(pats.size(), -1);
            for (size_t q = 0; q < sub.size(); q++) local[sub[q]] = (int)q;
            b.masks.resize((size_t)b.d.nstates * nchunks);
            for (int s = 0; s < b.d.nstates; s++) {
                uint64_t *m = &b.masks[(size_t)s * nchunks];
                for (size_t c = 0; c < nchunks; c++) m[c] = all[c];
                for (auto &rp : rm_pat) {
                    int q = local[rp.second];
                    if (q < 0) continue;  // checked by another DFA of this slot
                    bool acc = (b.d.accept[s][q >> 6] >> (q & 63)) & 1;
                    if (acc == pats[rp.second].invert) m[rp.first >> 6] &= ~bit(rp.first);
                }
            }
            built.push_back(std::move(b));
        }
    }
    if (built.size() > 255) { *err = "rule set needs more than 255 DFAs"; return -1; }
    if (nfas.size() > (size_t)kMaxNfaPerRuleset) { *err = "rule set needs more than 64 NFA matchers"; return -1; }
    H.nnfa = (uint8_t)nfas.size();
    H.ndfa = (uint8_t)built.size();
    // slot directory (built is ordered by slot)
    for (int s = 0, k = 0; s <= kNumSlots; s++) {
        while (k < (int)built.size() && built[k].slot < s) k++;
        H.slot_dfa[s] = (uint8_t)k;
    }

    // ---- assemble the image
    std::vector<uint8_t> img(sizeof(ImgHeader));
    std::vector<DevDfa> dd(built.size());
    H.dfa_off = Append(img, dd.data(), dd.size());
    H.init_off = Append(img, init.data(), init.size());
    H.absent_off = Append(img, absent.data(), absent.size());
    std::vector<int32_t> ids(nchunks * 64, -1);
    for (size_t r = 0; r < nr; r++) ids[r] = rules[r]->id;
    H.rule_off = Append(img, ids.data(), ids.size());
    std::vector<DevHdrName> hn;
    std::vector<uint8_t> names;
    for (auto &nm : custom) {
        DevHdrName h{};
        uint32_t hash = kFnvBasis;
        for (char c : nm) hash = l7_fnv_step(hash, (uint8_t)c);
        h.hash = hash;
        h.len = (uint16_t)nm.size();
        h.name_off = (uint32_t)names.size();
        names.insert(names.end(), nm.begin(), nm.end());
        hn.push_back(h);
    }
    {
        std::vector<DevNfaRef> refs(nfas.size());
        for (size_t k = 0; k < nfas.size(); k++) {
            refs[k].nfa = nfas[k].nfa;
            refs[k].slot = (uint8_t)nfas[k].slot;
            refs[k].mask_off = Append(img, nfas[k].masks.data(), nfas[k].masks.size());
        }
        H.nfa_off = Append(img, refs.data(), refs.size());
    }
    H.hdr_off = Append(img, hn.data(), hn.size());
    uint32_t names_off = Append(img, names.data(), names.size());
    for (auto &h : hn) h.name_off += names_off;
    if (!hn.empty()) memcpy(img.data() + H.hdr_off, hn.data(), hn.size() * sizeof(DevHdrName));
    {
        NameDfa nd = BuildNameDfa(custom);
        H.name_ncls = (uint16_t)nd.ncls;
        H.name_states = (uint16_t)nd.info.size();
        H.name_cls_off = Append(img, nd.cls, 256);
        H.name_trans_off = Append(img, nd.trans.data(), nd.trans.size());
        H.name_info_off = Append(img, nd.info.data(), nd.info.size());
        uint32_t bits = 0, mul = 0;
        const std::vector<DevNameEnt> tab = BuildNameTable(custom, &bits, &mul);
        H.ntab_bits = (uint8_t)bits;
        H.ntab_mul = mul;
        H.ntab_off = Append(img, tab.data(), tab.size());
    }
    for (size_t k = 0; k < built.size(); k++) {
        const re::DFA &d = built[k].d;
        dd[k].ncls = (uint16_t)d.ncls;
        dd[k].start = (uint16_t)d.start;
        dd[k].cls_off = Append(img, d.cls, 256);
        dd[k].trans_off = Append(img, d.next.data(), d.next.size());
        dd[k].mask_off = Append(img, built[k].masks.data(), built[k].masks.size());
        dd[k].absorb = built[k].absorb;
        H.total_states += (uint32_t)d.nstates;
    }
    memcpy(img.data() + H.dfa_off, dd.data(), dd.size() * sizeof(DevDfa));
    memcpy(img.data(), &H, sizeof H);
    img.resize((img.size() + 15) & ~(size_t)15);

    HttpImage &I = img_;
    DevRuleset rs{};
    rs.image_off = (uint32_t)I.images.size();
    rs.image_len = (uint32_t)img.size();
    if ((uint64_t)rs.image_off + img.size() > 0xFFFFFFFFull) { *err = "HTTP rule tables exceed 4 GiB"; return -1; }
    I.images.insert(I.images.end(), img.begin(), img.end());
    I.rulesets.push_back(rs);
    I.chunks += nchunks;
    I.dfas += built.size();
    I.dfa_states += H.total_states;
    return (int)I.rulesets.size() - 1;
}

}  // namespace l7
