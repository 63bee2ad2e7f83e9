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

private:
    const PolicySet *ps_;
    KafkaImage img_;
    std::unordered_map<std::string, int> topic_id_, client_id_;
    std::map<std::pair<std::vector<int>, int>, int> cache_;
    int Compile(const std::vector<const KafkaRule *> &rules, bool any);
};

uint32_t KafkaStrHash(const uint8_t *s, size_t n);

}  // namespace l7
