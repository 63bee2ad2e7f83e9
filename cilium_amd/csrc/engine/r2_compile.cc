#include "r2_compile.h"

#include <algorithm>
#include <cstring>
#include <functional>

#include "../regex/re_dfa.h"
#include "nfa_pool.h"

namespace l7 {

int R2Compiler::RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err) {
    std::vector<const R2Rule *> items;
    uint8_t terminal = V_DENY;  // no installed entry / policy not found => drop (instance.go:157-165)
    if (policy >= 0 && policy < (int)ps_->policies.size()) {
        const PortPolicy *ex, *wc;
        ps_->policies[policy].Lookup(ingress, port, &ex, &wc);
        bool decided = false;
        for (const PortPolicy *pp : {ex, wc}) {
            if (!pp || !pp->px_installed) continue;
            if (!pp->px_have_l7 || pp->rules.empty()) { terminal = V_ALLOW; decided = true; break; }  // :173-186
            for (auto &r : pp->rules) {
                if (!r.RemoteOk(remote)) continue;
                if (r.NumL7() == 0) { terminal = V_ALLOW; decided = true; break; }  // empty L7 set (:106-108)
                for (auto &m : r.r2) items.push_back(&m);  // other parsers' rules never match r2d2 data
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
}  // namespace

int R2Compiler::Compile(const std::vector<const R2Rule *> &rules, uint8_t terminal, std::string *err) {
    compiled++;
    const size_t nr = rules.size();
    if (nr > (size_t)kR2MaxChunks * 64) {
        *err = "r2d2 rule set has " + std::to_string(nr) + " rules (device limit " + std::to_string(kR2MaxChunks * 64) + ")";
        return -1;
    }
    const size_t nch = std::max<size_t>(1, (nr + 63) / 64);
    auto bit = [](size_t r) { return 1ull << (r & 63); };
    R2ImgHeader H{};
    H.nchunks = (uint8_t)nch;
    H.terminal = terminal;
    std::vector<uint64_t> cmd((size_t)R2_NCMD * nch, 0), nofile(nch, 0);
    std::vector<int> pats;  // rule index per regex pattern (one regex per rule)
    for (size_t r = 0; r < nr; r++) {
        for (int c = 0; c < R2_NCMD; c++)
            if (rules[r]->cmd < 0 || rules[r]->cmd == c) cmd[(size_t)c * nch + (r >> 6)] |= bit(r);
        if (rules[r]->file_re) pats.push_back((int)r);
        else nofile[r >> 6] |= bit(r);
    }
    // unanchored DFAs over the file regexes (regexp.MatchString), halving the
    // set until each fits; a regex over the budget on its own -> the NFA
    std::vector<std::vector<int>> parts;
    std::vector<re::DFA> dfas;
    std::vector<int> nfa_pats;
    std::function<bool(std::vector<int>)> build = [&](std::vector<int> sub) -> bool {
        std::vector<re::Pattern> ps;
        for (int q : sub) ps.push_back({rules[pats[q]]->file_re.get(), false});
        re::DFA d;
        std::string e;
        if (re::BuildDFA(ps, max_dfa_states, &d, &e)) { parts.push_back(sub); dfas.push_back(std::move(d)); return true; }
        if (sub.size() == 1) { nfa_pats.push_back(sub[0]); return true; }
        std::vector<int> a(sub.begin(), sub.begin() + sub.size() / 2), b(sub.begin() + sub.size() / 2, sub.end());
        return build(a) && build(b);
    };
    if (!pats.empty()) {
        std::vector<int> all;
        for (size_t q = 0; q < pats.size(); q++) all.push_back((int)q);
        if (!build(all)) return -1;
    }
    std::vector<std::pair<int, uint64_t>> nfas;  // (pattern, DevNfa offset)
    for (int q : nfa_pats) {
        const R2Rule &r = *rules[pats[q]];
        std::string e;
        auto it = nfa_cache_.find(r.file_src);
        if (it == nfa_cache_.end()) {
            re::BitNfa nf;
            if (re::BuildBitNfa({r.file_re.get(), false}, kNfaMaxWords * 64, &nf, &e)) {
                const uint64_t off = AppendDevNfa(nf, &img_.nfa_pool, err);
                if (off == ~0ull) return -1;
                it = nfa_cache_.emplace(r.file_src, off).first;
                img_.nfas++;
            }
        }
        if (it != nfa_cache_.end()) { nfas.emplace_back(q, it->second); continue; }
        re::DFA d;
        std::string e2, e3;
        // the large NFA (sparse rows, state sets in scratch) when one large DFA does not fit
        re::BitNfa nf;
        const bool big = re::BuildBitNfa({r.file_re.get(), false}, kNfaMaxPositions, &nf, &e3, kNfaMaxWords);
        if (!re::BuildDFA({{r.file_re.get(), false}}, big ? LargeNfaDfaBudget(nf.m, max_single_dfa_states) : max_single_dfa_states,
                          &d, &e2)) {
            if (!big) {
                *err = "r2d2 file regex too complex for the device (" + e3 + "): " + r.file_src;
                return -1;
            }
            const uint64_t off = AppendDevNfa(nf, &img_.nfa_pool, err);
            if (off == ~0ull) return -1;
            it = nfa_cache_.emplace(r.file_src, off).first;
            img_.nfas++;
            nfas.emplace_back(q, it->second);
            continue;
        }
        parts.push_back({q});
        dfas.push_back(std::move(d));
    }
    if (dfas.size() > 255 || nfas.size() > (size_t)kMaxNfaPerRuleset) { *err = "r2d2 rule set needs too many automata"; return -1; }
    H.ndfa = (uint8_t)dfas.size();
    H.nnfa = (uint8_t)nfas.size();

    std::vector<uint8_t> img(sizeof(R2ImgHeader));
    H.cmd_off = Append(img, cmd.data(), cmd.size());
    H.nofile_off = Append(img, nofile.data(), nofile.size());
    std::vector<int32_t> ids(nch * 64, -1);
    for (size_t r = 0; r < nr; r++) ids[r] = rules[r]->id;
    H.rule_off = Append(img, ids.data(), ids.size());
    std::vector<DevDfa> dd(dfas.size());
    H.dfa_off = Append(img, dd.data(), dd.size());
    {
        std::vector<DevNfaRef> refs(nfas.size());
        for (size_t k = 0; k < nfas.size(); k++) {
            std::vector<uint64_t> own(nch, 0);
            own[pats[nfas[k].first] >> 6] |= bit((size_t)pats[nfas[k].first]);
            refs[k].nfa = nfas[k].second;
            refs[k].mask_off = Append(img, own.data(), own.size());
        }
        H.nfa_off = Append(img, refs.data(), refs.size());
    }
    for (size_t k = 0; k < dfas.size(); k++) {
        const re::DFA &d = dfas[k];
        std::vector<uint64_t> masks((size_t)d.nstates * nch, 0);
        for (int s = 0; s < d.nstates; s++)
            for (size_t q = 0; q < parts[k].size(); q++)
                if ((d.accept[s][q >> 6] >> (q & 63)) & 1) {
                    const size_t r = (size_t)pats[parts[k][q]];
                    masks[(size_t)s * nch + (r >> 6)] |= bit(r);
                }
        dd[k].ncls = (uint16_t)d.ncls;
        dd[k].start = (uint16_t)d.start;
        dd[k].cls_off = Append(img, d.cls, 256);
        dd[k].trans_off = Append(img, d.next.data(), d.next.size());
        dd[k].mask_off = Append(img, masks.data(), masks.size());
        dd[k].absorb = (uint32_t)d.nstates;
    }
    if (!dd.empty()) memcpy(img.data() + H.dfa_off, dd.data(), dd.size() * sizeof(DevDfa));
    memcpy(img.data(), &H, sizeof H);
    img.resize((img.size() + 15) & ~(size_t)15);

    R2Image &I = img_;
    DevRuleset rs{};
    rs.image_off = (uint32_t)I.images.size();
    rs.image_len = (uint32_t)img.size();
    if ((uint64_t)rs.image_off + img.size() > 0xFFFFFFFFull) { *err = "r2d2 rule tables exceed 4 GiB"; return -1; }
    I.images.insert(I.images.end(), img.begin(), img.end());
    I.rulesets.push_back(rs);
    I.rules += nr;
    I.dfas += dfas.size();
    return (int)I.rulesets.size() - 1;
}

}  // namespace l7
