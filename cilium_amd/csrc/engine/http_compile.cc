#include "http_compile.h"

#include <algorithm>
#include <functional>
#include <memory>

#include "../regex/re_dfa.h"

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

int HttpCompiler::RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err) {
    std::vector<const HttpRule *> items;
    uint8_t terminal = V_DENY;
    if (policy >= 0 && policy < (int)ps_->policies.size()) {
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

int HttpCompiler::Compile(const std::vector<const HttpRule *> &rules, uint8_t terminal, std::string *err) {
    HttpImage &I = img_;
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

    DevRuleset rs{};
    rs.terminal = terminal;
    rs.nhdr = (uint8_t)custom.size();
    rs.hdr_first = (uint32_t)I.hdrs.size();
    for (auto &nm : custom) {
        DevHdrName h{};
        uint32_t hash = kFnvBasis;
        for (char c : nm) hash = l7_fnv_step(hash, (uint8_t)c);
        h.hash = hash;
        h.len = (uint16_t)nm.size();
        h.name_off = (uint32_t)I.names.size();
        I.names.insert(I.names.end(), nm.begin(), nm.end());
        I.hdrs.push_back(h);
    }
    rs.chunk_first = (uint32_t)I.chunks.size();

    for (size_t c0 = 0; c0 < rules.size() || (c0 == 0 && rules.empty()); c0 += 64) {
        if (rules.empty()) break;
        size_t c1 = std::min(rules.size(), c0 + 64);
        int nr = (int)(c1 - c0);
        DevChunk ch{};
        ch.nrules = (uint16_t)nr;
        ch.all_mask = nr == 64 ? ~0ull : ((1ull << nr) - 1);
        ch.rule_id_off = (uint32_t)I.rule_ids.size();
        for (size_t i = c0; i < c1; i++) I.rule_ids.push_back(rules[i]->id);
        ch.field_first = (uint32_t)I.fields.size();

        // matchers grouped by slot: (rule index in chunk, matcher)
        std::map<int, std::vector<std::pair<int, const HeaderMatcher *>>> by_slot;
        for (size_t i = c0; i < c1; i++)
            for (auto &m : rules[i]->m) by_slot[slot_of(m.name)].emplace_back((int)(i - c0), &m);

        for (auto &kv : by_slot) {
            DevField f{};
            f.slot = (uint8_t)kv.first;
            uint64_t constrained = 0;
            for (auto &rm : kv.second) constrained |= 1ull << rm.first;
            f.absent_mask = ch.all_mask & ~constrained;
            f.dfa_first = (uint32_t)I.dfas.size();
            if (kv.first == kSlotNever) { f.ndfa = 0; I.fields.push_back(f); continue; }

            // distinct patterns of this field
            std::vector<Pat> pats;
            std::vector<std::pair<int, int>> rm_pat;  // (rule, pattern)
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
            // build DFAs, halving the pattern set until each fits the budget
            std::vector<std::vector<int>> groups;
            std::vector<re::DFA> dfas;
            std::function<bool(std::vector<int>)> build = [&](std::vector<int> sub) -> bool {
                std::vector<re::Pattern> ps;
                for (int p : sub) ps.push_back({asts[p], true});
                re::DFA d;
                std::string e;
                if (re::BuildDFA(ps, max_dfa_states, &d, &e)) { groups.push_back(sub); dfas.push_back(std::move(d)); return true; }
                if (sub.size() == 1) { *err = "regex too complex for the DFA budget: " + pats[sub[0]].value; return false; }
                std::vector<int> a(sub.begin(), sub.begin() + sub.size() / 2), b(sub.begin() + sub.size() / 2, sub.end());
                return build(a) && build(b);
            };
            std::vector<int> all;
            for (size_t p = 0; p < pats.size(); p++) all.push_back((int)p);
            if (!build(all)) return -1;
            if (dfas.size() > 255) { *err = "too many DFAs for one header field"; return -1; }
            f.ndfa = (uint8_t)dfas.size();
            for (size_t g = 0; g < dfas.size(); g++) {
                const re::DFA &d = dfas[g];
                const std::vector<int> &sub = groups[g];
                DevDfa dd{};
                dd.trans_off = (uint32_t)I.trans.size();
                dd.mask_off = (uint32_t)I.masks.size();
                dd.cls_off = (uint32_t)I.cls.size();
                dd.ncls = (uint16_t)d.ncls;
                dd.start = (uint16_t)d.start;
                I.cls.insert(I.cls.end(), d.cls, d.cls + 256);
                I.trans.insert(I.trans.end(), d.next.begin(), d.next.end());
                for (int s = 0; s < d.nstates; s++) {
                    uint64_t mask = ch.all_mask;
                    for (auto &rp : rm_pat) {
                        auto pos = std::find(sub.begin(), sub.end(), rp.second);
                        if (pos == sub.end()) continue;  // checked by another DFA of this field
                        int local = (int)(pos - sub.begin());
                        bool acc = (d.accept[s][local >> 6] >> (local & 63)) & 1;
                        if (acc == pats[rp.second].invert) mask &= ~(1ull << rp.first);
                    }
                    I.masks.push_back(mask);
                }
                I.dfa_states += d.nstates;
                I.dfas.push_back(dd);
            }
            I.fields.push_back(f);
        }
        ch.nfields = (uint16_t)(I.fields.size() - ch.field_first);
        I.chunks.push_back(ch);
    }
    rs.nchunks = (uint16_t)(I.chunks.size() - rs.chunk_first);
    I.rulesets.push_back(rs);
    return (int)I.rulesets.size() - 1;
}

}  // namespace l7
