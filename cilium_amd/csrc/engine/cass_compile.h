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
#include "../policy/policy.h"

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
    explicit CassCompiler(const PolicySet *ps);
    // remote = the connection's source identity (connection.go:176-179)
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t remote, std::string *err);
    const CassImage &image() const { return img_; }
    int max_dfa_states = 4096;
    int max_single_dfa_states = 65535;

private:
    const PolicySet *ps_;
    CassImage img_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    std::map<std::string, uint64_t> nfa_cache_;
    int Compile(const std::vector<const CassRule *> &rules, uint8_t terminal, std::string *err);
};

}  // namespace l7
