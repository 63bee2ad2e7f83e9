// memcached rule-set compiler (product code): proxylib's memcache policy
// semantics lowered to device tables (device_tables.h McImgHeader).
//
// For a connection (policy, direction, port, source identity) proxylib
// evaluates PortNetworkPolicies.Matches (proxylib/proxylib/policymap.go:210-236):
// the exact-port entry, then the port-0 entry, each only if installed (every
// rule's parser registered, :113-148).  An entry without L7 rules allows; a
// rule group admitting the identity with no L7 rules allows; otherwise the
// group's memcache.Rule list is tried in order.  That order is fixed per
// connection, so it is resolved here once into a rule set: the ordered rule
// list up to the first unconditional allow + the terminal verdict.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <vector>

#include "../device_tables.h"
#include "nfa_pool.h"
#include "../policy/policy.h"
#include "serial.h"

namespace l7 {

struct McImage {
    std::vector<DevRuleset> rulesets;
    std::vector<uint8_t> images;
    std::vector<uint8_t> nfa_pool;  // DevNfa tables of keyRegex patterns over the DFA budget
    size_t rules = 0, dfas = 0, dfa_states = 0, nfas = 0;
    size_t max_chunks = 0;  // most 64-rule chunks of any rule set (selects the kernel instantiation)
};

class McCompiler {
public:
    // the largest state set (u64 words) among its NFAs (large ones: > kNfaMaxWords)
    uint32_t nfa_max_words() const { return NfaPoolMaxWords(img_.nfa_pool, nfa_cache_); }
    explicit McCompiler(const PolicySet *ps) : ps_(ps) {}
    // remote = the connection's source identity (proxylib/proxylib/connection.go:176-179)
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err);
    const McImage &image() const { return img_; }
    int max_dfa_states = 4096;
    int max_single_dfa_states = 65535;  // a pattern the NFA cannot take (see HttpCompiler)

    // compiled state of this policy version (engine/serial.h): written by the
    // rank that compiled it, installed by the others without compiling
    void Save(Ser &s) const {
        s.vec(img_.rulesets); s.vec(img_.images); s.vec(img_.nfa_pool);
        s.cache(cache_); s.smap(nfa_cache_);
        s.u64(img_.rules); s.u64(img_.dfas); s.u64(img_.dfa_states); s.u64(img_.nfas); s.u64(img_.max_chunks);
    }
    bool Load(Des &d) {
        d.vec(img_.rulesets); d.vec(img_.images); d.vec(img_.nfa_pool);
        d.cache(cache_); d.smap(nfa_cache_);
        img_.rules = d.u64(); img_.dfas = d.u64(); img_.dfa_states = d.u64(); img_.nfas = d.u64();
        img_.max_chunks = d.u64();
        return d.ok && NfaOffsetsValid(img_.nfa_pool, nfa_cache_) && RulesetImagesValid(img_.rulesets, img_.images) &&
               ImageNfaRefsValid<McImgHeader>(img_.rulesets, img_.images, nfa_cache_, 8);
    }
    size_t compiled = 0;  // rule sets compiled (not taken from the cache) since construction

private:
    const PolicySet *ps_;
    McImage img_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    std::map<std::string, uint64_t> nfa_cache_;  // keyRegex -> DevNfa offset in the pool
    int Compile(const std::vector<const McRule *> &rules, uint8_t terminal, std::string *err);
};

}  // namespace l7
