// r2d2 rule-set compiler (product code): proxylib's r2d2 policy semantics
// (proxylib/r2d2/r2d2parser.go:31-107 + the proxylib policymap,
// proxylib/proxylib/policymap.go:91-236) lowered to R2ImgHeader images.
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

struct R2Image {
    std::vector<DevRuleset> rulesets;
    std::vector<uint8_t> images;
    std::vector<uint8_t> nfa_pool;
    size_t rules = 0, dfas = 0, nfas = 0;
};

class R2Compiler {
public:
    // the largest state set (u64 words) among its NFAs (large ones: > kNfaMaxWords)
    uint32_t nfa_max_words() const { return NfaPoolMaxWords(img_.nfa_pool, nfa_cache_); }
    explicit R2Compiler(const PolicySet *ps) : ps_(ps) {}
    // remote = the connection's source identity (connection.go:176-179)
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err);
    const R2Image &image() const { return img_; }
    int max_dfa_states = 4096;
    int max_single_dfa_states = 65535;

    // compiled state of this policy version (engine/serial.h): written by the
    // rank that compiled it, installed by the others without compiling
    void Save(Ser &s) const {
        s.vec(img_.rulesets); s.vec(img_.images); s.vec(img_.nfa_pool);
        s.cache(cache_); s.smap(nfa_cache_);
        s.u64(img_.rules); s.u64(img_.dfas); s.u64(img_.nfas);
    }
    bool Load(Des &d) {
        d.vec(img_.rulesets); d.vec(img_.images); d.vec(img_.nfa_pool);
        d.cache(cache_); d.smap(nfa_cache_);
        img_.rules = d.u64(); img_.dfas = d.u64(); img_.nfas = d.u64();
        return d.ok && NfaOffsetsValid(img_.nfa_pool, nfa_cache_) && RulesetImagesValid(img_.rulesets, img_.images) &&
               ImageNfaRefsValid<R2ImgHeader>(img_.rulesets, img_.images, nfa_cache_, 8);
    }
    size_t compiled = 0;  // rule sets compiled (not taken from the cache) since construction

private:
    const PolicySet *ps_;
    R2Image img_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    std::map<std::string, uint64_t> nfa_cache_;
    int Compile(const std::vector<const R2Rule *> &rules, uint8_t terminal, std::string *err);
};

}  // namespace l7
