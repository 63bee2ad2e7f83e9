#include "mc_compile.h"

#include <algorithm>
#include <cstring>
#include <functional>
#include <memory>

#include "../regex/re_dfa.h"
#include "mc_groups.h"
#include "nfa_pool.h"

namespace l7 {

int McCompiler::RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err) {
    std::vector<const McRule *> items;
    uint8_t terminal = V_DENY;  // no installed entry / policy not found => drop (instance.go:157-165)
    if (policy >= 0 && policy < (int)ps_->policies.size()) {
        const PortPolicy *ex, *wc;
        ps_->policies[policy].Lookup(ingress, port, &ex, &wc);
        bool decided = false;
        for (const PortPolicy *pp : {ex, wc}) {
            if (!pp || !pp->px_installed) continue;
            // !HaveL7Rules or no rules at all: matches (policymap.go:173-186)
            if (!pp->px_have_l7 || pp->rules.empty()) { terminal = V_ALLOW; decided = true; break; }
            for (auto &r : pp->rules) {
                if (!r.RemoteOk(remote)) continue;
                if (r.NumL7() == 0) { terminal = V_ALLOW; decided = true; break; }  // empty L7 set (:106-108)
                for (auto &m : r.mc) items.push_back(&m);  // HTTP / Kafka rules never match a memcached request
            }
            if (decided) break;
        }
    }
    std::vector<int> ids;
    for (auto *m : items) ids.push_back(m->id);
    auto key = std::make_pair(ids, (int)terminal);
    auto it = cache_.find(key);
    if (it != cache_.end()) return it->second;
    int rs = Compile(items, terminal, err);
    if (rs >= 0) cache_.emplace(key, rs);
    return rs;
}

namespace {

template <class T>
uint32_t Append(std::vector<uint8_t> &img, const T *p, size_t n) {
    size_t off = (img.size() + 15) & ~(size_t)15;
    img.resize(off + n * sizeof(T));
    if (n) memcpy(img.data() + off, p, n * sizeof(T));
    return (uint32_t)off;
}

// keyExact: bytes.Equal; keyPrefix: bytes.HasPrefix — raw byte semantics, so
// they are built from the byte ops of the DFA compiler and matched anchored.
std::unique_ptr<re::Node> LiteralAst(const std::string &v, bool prefix) {
    auto b = std::make_unique<re::Node>(re::Op::ByteString);
    b->bytes = v;
    if (!prefix) return b;
    auto c = std::make_unique<re::Node>(re::Op::Concat);
    c->sub.push_back(std::move(b));
    c->sub.push_back(std::make_unique<re::Node>(re::Op::AnyBytes));
    return c;
}

}  // namespace

int McCompiler::Compile(const std::vector<const McRule *> &rules, uint8_t terminal, std::string *err) {
    compiled++;
    const size_t nr = rules.size();
    if (nr > (size_t)kMcMaxChunks * 64) {
        *err = "memcache rule set has " + std::to_string(nr) + " rules (device limit " + std::to_string(kMcMaxChunks * 64) + ")";
        return -1;
    }
    const size_t nch = std::max<size_t>(1, (nr + 63) / 64);
    auto bit = [](size_t r) { return 1ull << (r & 63); };
    McImgHeader H{};
    H.nchunks = (uint8_t)nch;
    H.terminal = terminal;

    int ngroups;
    const McGroup *groups = McGroups(&ngroups);
    std::vector<uint64_t> text((size_t)kMcTextRows * nch, 0), ops((size_t)256 * nch, 0), empty(nch, 0), nopred(nch, 0);
    // key predicates: (rule, pattern) with the effective predicate of Rule.Matches
    struct Pat { std::unique_ptr<re::Node> own; const re::Node *ast; bool anchored; std::string src; };
    std::vector<Pat> pats;
    std::vector<std::pair<size_t, int>> rule_pat;
    for (size_t r = 0; r < nr; r++) {
        const McRule &m = *rules[r];
        if (m.empty) { empty[r >> 6] |= bit(r); continue; }
        const McGroup &g = groups[m.group];
        for (int t = 0; t < kMcTextIds; t++)
            if ((g.text >> t) & 1) text[(size_t)t * nch + (r >> 6)] |= bit(r);
        for (int k = 0; k < g.nops; k++) ops[(size_t)g.ops[k] * nch + (r >> 6)] |= bit(r);
        if (!m.key_exact.empty()) {
            auto a = LiteralAst(m.key_exact, false);
            const re::Node *p = a.get();
            pats.push_back({std::move(a), p, true});
        } else if (!m.key_prefix.empty()) {
            auto a = LiteralAst(m.key_prefix, true);
            const re::Node *p = a.get();
            pats.push_back({std::move(a), p, true});
        } else if (m.key_re) {
            pats.push_back({nullptr, m.key_re.get(), false, m.key_re_src});  // regexp.Match: unanchored
        } else {
            nopred[r >> 6] |= bit(r);
            continue;
        }
        rule_pat.emplace_back(r, (int)pats.size() - 1);
    }

    // DFAs over the key predicates, halving the pattern set until each fits
    std::vector<std::vector<int>> parts;
    std::vector<re::DFA> dfas;
    std::vector<int> nfa_pats;
    std::function<bool(std::vector<int>)> build = [&](std::vector<int> sub) -> bool {
        std::vector<re::Pattern> ps;
        for (int p : sub) ps.push_back({pats[p].ast, pats[p].anchored});
        re::DFA d;
        std::string e;
        if (re::BuildDFA(ps, max_dfa_states, &d, &e)) { parts.push_back(sub); dfas.push_back(std::move(d)); return true; }
        if (sub.size() == 1) { nfa_pats.push_back(sub[0]); return true; }  // over the budget alone: the NFA
        std::vector<int> a(sub.begin(), sub.begin() + sub.size() / 2), b(sub.begin() + sub.size() / 2, sub.end());
        return build(a) && build(b);
    };
    if (!pats.empty()) {
        std::vector<int> allp;
        for (size_t p = 0; p < pats.size(); p++) allp.push_back((int)p);
        if (!build(allp)) return -1;
    }
    std::vector<std::pair<int, uint64_t>> nfas;  // (pattern, DevNfa offset)
    for (int p : nfa_pats) {
        std::string e;
        auto it = nfa_cache_.find(pats[p].src);
        if (it == nfa_cache_.end() && !pats[p].anchored) {
            re::BitNfa nf;
            if (re::BuildBitNfa({pats[p].ast, false}, kNfaMaxWords * 64, &nf, &e)) {
                const uint64_t off = AppendDevNfa(nf, &img_.nfa_pool, err);
                if (off == ~0ull) return -1;
                it = nfa_cache_.emplace(pats[p].src, off).first;
                img_.nfas++;
            }
        }
        if (it != nfa_cache_.end()) {
            nfas.emplace_back(p, it->second);
            continue;
        }
        re::DFA d;
        std::string e2, e3;
        // the large NFA (sparse rows, state sets in scratch) when one large DFA does not fit
        re::BitNfa nf;
        const bool big = !pats[p].anchored && re::BuildBitNfa({pats[p].ast, false}, kNfaMaxPositions, &nf, &e3, kNfaMaxWords);
        if (!re::BuildDFA({{pats[p].ast, pats[p].anchored}},
                          big ? LargeNfaDfaBudget(nf.m, max_single_dfa_states) : max_single_dfa_states, &d, &e2)) {
            if (!big) {
                *err = "memcache key pattern too complex for the device (" + (e3.empty() ? e2 : e3) + "): " + pats[p].src;
                return -1;
            }
            const uint64_t off = AppendDevNfa(nf, &img_.nfa_pool, err);
            if (off == ~0ull) return -1;
            it = nfa_cache_.emplace(pats[p].src, off).first;
            img_.nfas++;
            nfas.emplace_back(p, it->second);
            continue;
        }
        parts.push_back({p});
        dfas.push_back(std::move(d));
    }
    if (dfas.size() > 255) { *err = "memcache key patterns need more than 255 DFAs"; return -1; }
    if (nfas.size() > (size_t)kMaxNfaPerRuleset) { *err = "memcache rule set needs more than 64 NFA matchers"; return -1; }
    H.ndfa = (uint8_t)dfas.size();

    std::vector<uint8_t> img(sizeof(McImgHeader));
    // the DFA descriptors first, at kMcDfaOff: the kernel's key-byte step then
    // reads them at a constant offset instead of through the header
    std::vector<DevDfa> dd(dfas.size());
    H.dfa_off = Append(img, dd.data(), dd.size());
    if (H.dfa_off != kMcDfaOff) { *err = "memcache image layout"; return -1; }
    H.text_off = Append(img, text.data(), text.size());
    H.op_off = Append(img, ops.data(), ops.size());
    H.empty_off = Append(img, empty.data(), empty.size());
    H.nopred_off = Append(img, nopred.data(), nopred.size());
    std::vector<int32_t> ids(nch * 64, -1);
    for (size_t r = 0; r < nr; r++) ids[r] = rules[r]->id;
    H.rule_off = Append(img, ids.data(), ids.size());
    std::vector<uint64_t> owned(dfas.size() * nch, 0);
    for (size_t k = 0; k < dfas.size(); k++)
        for (auto &rp : rule_pat)
            if (std::find(parts[k].begin(), parts[k].end(), rp.second) != parts[k].end())
                owned[k * nch + (rp.first >> 6)] |= bit(rp.first);
    H.owned_off = Append(img, owned.data(), owned.size());
    {
        std::vector<DevNfaRef> refs(nfas.size());
        for (size_t k = 0; k < nfas.size(); k++) {
            std::vector<uint64_t> own(nch, 0);
            for (auto &rp : rule_pat)
                if (rp.second == nfas[k].first) own[rp.first >> 6] |= bit(rp.first);
            refs[k].nfa = nfas[k].second;
            refs[k].mask_off = Append(img, own.data(), own.size());
        }
        H.nfa_off = Append(img, refs.data(), refs.size());
        H.nnfa = (uint32_t)nfas.size();
    }
    size_t states = 0;
    for (size_t k = 0; k < dfas.size(); k++) {
        const re::DFA &d = dfas[k];
        std::vector<int> local(pats.size(), -1);
        for (size_t q = 0; q < parts[k].size(); q++) local[parts[k][q]] = (int)q;
        std::vector<uint64_t> masks((size_t)d.nstates * nch, 0);
        for (int s = 0; s < d.nstates; s++)
            for (auto &rp : rule_pat) {
                int q = local[rp.second];
                if (q >= 0 && ((d.accept[s][q >> 6] >> (q & 63)) & 1)) masks[(size_t)s * nch + (rp.first >> 6)] |= bit(rp.first);
            }
        dd[k].ncls = (uint16_t)d.ncls;
        dd[k].start = (uint16_t)d.start;
        dd[k].cls_off = Append(img, d.cls, 256);
        dd[k].trans_off = Append(img, d.next.data(), d.next.size());
        dd[k].mask_off = Append(img, masks.data(), masks.size());
        dd[k].absorb = (uint32_t)d.nstates;  // (unused by the memcached kernel)
        states += (size_t)d.nstates;
    }
    if (!dd.empty()) memcpy(img.data() + H.dfa_off, dd.data(), dd.size() * sizeof(DevDfa));
    memcpy(img.data(), &H, sizeof H);
    img.resize((img.size() + 15) & ~(size_t)15);

    McImage &I = img_;
    DevRuleset rs{};
    rs.image_off = (uint32_t)I.images.size();
    rs.image_len = (uint32_t)img.size();
    if ((uint64_t)rs.image_off + img.size() > 0xFFFFFFFFull) { *err = "memcache rule tables exceed 4 GiB"; return -1; }
    I.images.insert(I.images.end(), img.begin(), img.end());
    I.rulesets.push_back(rs);
    I.rules += nr;
    I.max_chunks = std::max(I.max_chunks, nch);
    I.dfas += dfas.size();
    I.dfa_states += states;
    return (int)I.rulesets.size() - 1;
}

}  // namespace l7
