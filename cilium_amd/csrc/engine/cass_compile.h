// cassandra rule-set compiler (product code): proxylib's cassandra policy
// semantics (proxylib/cassandra/cassandraparser.go:50-134 + the proxylib
// policymap, proxylib/proxylib/policymap.go:91-236) lowered to CassImgHeader
// images.
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

struct CassImage {
    std::vector<DevRuleset> rulesets;
    std::vector<uint8_t> images;
    std::vector<uint8_t> nfa_pool;
    std::vector<uint32_t> lower;  // unicode.ToLower pairs (rune, lower), flattened
    size_t rules = 0, dfas = 0, nfas = 0;
};

class CassCompiler {
public:
    // the largest state set (u64 words) among its NFAs (large ones: > kNfaMaxWords)
    uint32_t nfa_max_words() const { return NfaPoolMaxWords(img_.nfa_pool, nfa_cache_); }
    explicit CassCompiler(const PolicySet *ps);
    // remote = the connection's source identity (connection.go:176-179)
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err);
    const CassImage &image() const { return img_; }
    int max_dfa_states = 4096;
    int max_single_dfa_states = 65535;

    // compiled state of this policy version (engine/serial.h): written by the
    // rank that compiled it, installed by the others without compiling
    void Save(Ser &s) const {
        s.vec(img_.rulesets); s.vec(img_.images); s.vec(img_.nfa_pool);
        s.cache(cache_); s.smap(nfa_cache_);
        s.vec(img_.lower); s.u64(img_.rules); s.u64(img_.dfas); s.u64(img_.nfas);
    }
    bool Load(Des &d) {
        d.vec(img_.rulesets); d.vec(img_.images); d.vec(img_.nfa_pool);
        d.cache(cache_); d.smap(nfa_cache_);
        d.vec(img_.lower); img_.rules = d.u64(); img_.dfas = d.u64(); img_.nfas = d.u64();
        return d.ok && NfaOffsetsValid(img_.nfa_pool, nfa_cache_) && RulesetImagesValid(img_.rulesets, img_.images) &&
               ImageNfaRefsValid<CassImgHeader>(img_.rulesets, img_.images, nfa_cache_, 8);
    }
    size_t compiled = 0;  // rule sets compiled (not taken from the cache) since construction

private:
    const PolicySet *ps_;
    CassImage img_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    std::map<std::string, uint64_t> nfa_cache_;
    int Compile(const std::vector<const CassRule *> &rules, uint8_t terminal, std::string *err);
};

}  // namespace l7
