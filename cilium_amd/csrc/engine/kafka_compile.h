// Kafka rule-set compiler (product code).
//
// The relevant rules for a connection are GetRelevantRules(source identity)
// (pkg/policy/l4.go:118-141): every group (PortNetworkPolicyRule) of the
// port entry whose remote set admits the identity contributes its Kafka rules
// in order; an L3-only group contributes the L7 wildcard rule {} (the L3
// override of pkg/policy/repository.go:135-160).  No contributing group =>
// rules.Kafka == nil => deny (pkg/proxy/kafka.go:139-142).
//
// MatchesRule (pkg/kafka/policy.go:200-225) is evaluated on the device from
// three precomputed views of the ordered rule list:
//   topicless : positions of rules with Topic == ""
//   per topic : for each topic id, the positions of rules naming it
//   per key   : for each api key, the positions of rules whose key set admits it
// Verdict = first position among {first matching topicless rule,
// max over request topics of the first matching rule of that topic}.
#pragma once
#include <cstdint>
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

#include "../device_tables.h"
#include "../policy/policy.h"
#include "serial.h"

namespace l7 {

struct KafkaImage {
    std::vector<DevKafkaRuleset> rulesets;
    std::vector<DevKafkaRule> rules;
    std::vector<uint32_t> index;
    std::vector<DevStrSlot> topic_hash, client_hash;
    std::vector<uint8_t> strings;
    uint32_t topic_mask = 0, client_mask = 0;
    size_t ntopics = 0;
};

class KafkaCompiler {
public:
    explicit KafkaCompiler(const PolicySet *ps);
    // proxylib: the proxylib "kafka" parser's view of the port entries
    int RulesetFor(int policy, bool ingress, uint32_t port, uint64_t src_id, bool proxylib, std::string *err);
    const KafkaImage &image() const { return img_; }

    // compiled state of this policy version (engine/serial.h): written by the
    // rank that compiled it, installed by the others without compiling
    void Save(Ser &s) const {
        s.vec(img_.rulesets); s.vec(img_.rules); s.vec(img_.index); s.vec(img_.topic_hash); s.vec(img_.client_hash);
        s.vec(img_.strings); s.u64(img_.topic_mask); s.u64(img_.client_mask); s.u64(img_.ntopics);
        s.umap(topic_id_); s.umap(client_id_); s.cache(cache_);
    }
    bool Load(Des &d) {
        d.vec(img_.rulesets); d.vec(img_.rules); d.vec(img_.index); d.vec(img_.topic_hash); d.vec(img_.client_hash);
        d.vec(img_.strings); img_.topic_mask = (uint32_t)d.u64(); img_.client_mask = (uint32_t)d.u64();
        img_.ntopics = d.u64();
        d.umap(topic_id_); d.umap(client_id_); d.cache(cache_);
        // the kernels probe the hash tables with the masks and read rules by index
        auto table_ok = [](const std::vector<DevStrSlot> &t, uint32_t mask) {
            return !t.empty() && (uint64_t)mask + 1 == t.size() && (t.size() & (t.size() - 1)) == 0;
        };
        if (!d.ok || !table_ok(img_.topic_hash, img_.topic_mask) || !table_ok(img_.client_hash, img_.client_mask))
            return false;
        for (const auto &r : img_.rulesets)
            if ((uint64_t)r.rule_first + r.nrules > img_.rules.size()) return false;
        return true;
    }
    size_t compiled = 0;  // rule sets compiled (not taken from the cache) since construction

private:
    const PolicySet *ps_;
    KafkaImage img_;
    std::unordered_map<std::string, int> topic_id_, client_id_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    int Compile(const std::vector<const KafkaRule *> &rules, bool any);
};

uint32_t KafkaStrHash(const uint8_t *s, size_t n);

}  // namespace l7
