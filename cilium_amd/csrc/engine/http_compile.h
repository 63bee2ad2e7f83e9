// HTTP rule-set compiler (product code): Envoy HTTP policy semantics
// (envoy/cilium_network_policy.h:50-237) lowered to device tables.
//
// For a connection (policy, direction, port, remote identity) the verdict is
// the first HTTP rule, in PortNetworkPolicy evaluation order, whose header
// matchers all match; the order is fixed per connection, so it is resolved
// here once into a "rule set": an ordered rule list + a terminal verdict.
// Each rule set becomes one self-contained image (device_tables.h): rules in
// chunks of <= 64, and per header slot the matchers of ALL rules compiled
// into byte DFAs whose states carry, per chunk, the mask of rules satisfied
// on that slot if the value ends there.  The kernel walks these DFAs while it
// frames the request, so every request byte is read once.
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

struct HttpImage {
    std::vector<DevRuleset> rulesets;
    std::vector<uint8_t> images;
    std::vector<uint8_t> nfa_pool;  // DevNfa tables (device_tables.h), shared by all rule sets
    size_t chunks = 0, dfas = 0, dfa_states = 0, nfas = 0;
};

class HttpCompiler {
public:
    // the largest state set (u64 words) among its NFAs (large ones: > kNfaMaxWords)
    uint32_t nfa_max_words() const { return NfaPoolMaxWords(img_.nfa_pool, nfa_cache_); }
    explicit HttpCompiler(const PolicySet *ps) : ps_(ps) {}
    // Returns the rule set index for a connection, compiling it on first use.
    // policy < 0: unknown policy (NetworkPolicyMap::Allowed => deny).
    // proxylib: the proxylib "http" parser's policymap semantics (no port entry
    // => drop, installed entries only) instead of Envoy's NetworkPolicyMap
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, bool proxylib, std::string *err);
    const HttpImage &image() const { return img_; }
    int max_dfa_states = 4096;
    // A pattern whose DFA alone exceeds max_dfa_states is evaluated by the
    // bit-parallel NFA (<= kNfaMaxWords * 64 positions), else by one DFA of up
    // to max_single_dfa_states; beyond both the policy is rejected.
    int max_single_dfa_states = 65535;

    // compiled state of this policy version (engine/serial.h): written by the
    // rank that compiled it, installed by the others without compiling
    void Save(Ser &s) const {
        s.vec(img_.rulesets); s.vec(img_.images); s.vec(img_.nfa_pool);
        s.cache(cache_); s.smap(nfa_cache_);
        s.u64(img_.chunks); s.u64(img_.dfas); s.u64(img_.dfa_states); s.u64(img_.nfas);
    }
    bool Load(Des &d) {
        d.vec(img_.rulesets); d.vec(img_.images); d.vec(img_.nfa_pool);
        d.cache(cache_); d.smap(nfa_cache_);
        img_.chunks = d.u64(); img_.dfas = d.u64(); img_.dfa_states = d.u64(); img_.nfas = d.u64();
        return d.ok && NfaOffsetsValid(img_.nfa_pool, nfa_cache_) && RulesetImagesValid(img_.rulesets, img_.images) &&
               ImageNfaRefsValid<ImgHeader>(img_.rulesets, img_.images, nfa_cache_, 16);
    }
    size_t compiled = 0;  // rule sets compiled (not taken from the cache) since construction

private:
    const PolicySet *ps_;
    HttpImage img_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;  // (rule ids, terminal) -> ruleset
    std::map<std::string, uint64_t> nfa_cache_;              // regex -> DevNfa offset in the pool
    int Compile(const std::vector<const HttpRule *> &rules, uint8_t terminal, std::string *err);
};

}  // namespace l7
