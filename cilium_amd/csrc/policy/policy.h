// L7 policy model (product code): the NPDS cilium.NetworkPolicy shape
// (envoy/cilium/npds.proto:31-182) with the reference's rule types:
//   HTTP  : HttpNetworkPolicyRule = AND of Envoy HeaderMatchers, produced from
//           api.PortRuleHTTP by getHTTPRule (pkg/envoy/server.go:336-399)
//   Kafka : api.PortRuleKafka + Sanitize (pkg/policy/api/kafka.go:26-293,
//           rule_validation.go:232-275)
//   L7    : generic key/value rules for proxylib parsers (npds.proto:179-182)
#pragma once
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../regex/re_ast.h"

namespace l7 {

enum class HM : uint8_t { Exact, Regex, Present, Prefix, Suffix, Range };

struct HeaderMatcher {
    std::string name;   // lower-cased (Envoy LowerCaseString)
    HM type = HM::Exact;
    std::string value;
    bool invert = false;
    int64_t rstart = 0, rend = 0;
    std::shared_ptr<re::Node> ast;  // HM::Regex
};

struct HttpRule { std::vector<HeaderMatcher> m; int id = -1; };

struct KafkaRule {
    uint64_t keymask = 0;  // api keys 0..63
    bool any_key = true;   // apiKeyInt empty (CheckAPIKeyRole wildcard)
    bool has_version = false;
    int16_t version = 0;
    std::string topic, client;
    int id = -1;
};

struct L7Rule { std::vector<std::pair<std::string, std::string>> kv; int id = -1; };

// memcache.Rule (proxylib/memcached/parser.go:35-44), parsed by the loader
// from an l7_proto "memcache" rule's key/value map (parser.go:114-148).
struct McRule {
    int group = -1;          // MemcacheOpCodeMap entry (engine/mc_groups.h), -1 = none
    std::string key_exact, key_prefix;
    std::shared_ptr<re::Node> key_re;
    std::string key_re_src;
    bool empty = false;      // no command and no key: matches every request
    int id = -1;
};

// r2d2.R2d2Rule (proxylib/r2d2/r2d2parser.go:31-67): cmd exact (one of READ
// WRITE HALT RESET, or any), file regex (unanchored MatchString, or any).
enum : int { R2_READ = 0, R2_WRITE = 1, R2_HALT = 2, R2_RESET = 3, R2_OTHER = 4, R2_NCMD = 5 };
struct R2Rule {
    int cmd = -1;            // R2_* or -1 = any command
    std::shared_ptr<re::Node> file_re;
    std::string file_src;
    int id = -1;
};

// cassandra.CassandraRule (proxylib/cassandra/cassandraparser.go:50-53):
// query_action exact (an action id of kernels/cass_parse.h, -1 = any) and a
// query_table regex (unanchored MatchString, or any).
struct CassRule {
    int action = -1;
    std::shared_ptr<re::Node> table_re;
    std::string table_src;
    int id = -1;
};

struct PortRule {
    std::vector<uint64_t> remotes;  // empty = any remote
    enum Type { None, Http, Kafka, L7 } type = None;
    std::vector<HttpRule> http;
    std::vector<KafkaRule> kafka;
    std::string l7proto;
    std::vector<L7Rule> l7;
    std::vector<McRule> mc;  // l7proto == "memcache": its parsed L7 rules
    std::vector<R2Rule> r2;  // l7proto == "r2d2": its parsed L7 rules
    std::vector<CassRule> cass;  // l7proto == "cassandra": its parsed L7 rules
    size_t other_l7 = 0;     // "test.headerparser" rules (registered; never match here)
    // proxylib parser name: l7_proto, else the oneof type name, "" = no L7
    // (proxylib/proxylib/policymap.go:68-75)
    std::string ParserName() const;
    bool RemoteOk(uint64_t id) const;
    // parsed L7 rules of this group (proxylib's len(L7Rules)): memcache rules,
    // HTTP rules or Kafka rules
    size_t NumL7() const {
        return type == Http ? http.size() : type == Kafka ? kafka.size() : l7proto == "r2d2" ? r2.size()
             : l7proto == "memcache" ? mc.size() : l7proto == "cassandra" ? cass.size() : other_l7;
    }
};
// L7 rule parsers the proxylib view registers (policymap.go:42-45): "memcache",
// "r2d2", "cassandra", "test.headerparser", "PortNetworkPolicyRule_HttpRules",
// "PortNetworkPolicyRule_KafkaRules".
bool ProxylibParserRegistered(const std::string &name);

struct PortPolicy {
    uint32_t port = 0;
    bool tcp = true;
    std::vector<PortRule> rules;
    bool has_http = false;
    // proxylib view (policymap.go:113-148): the entry is installed only if every
    // rule's parser up to the first unregistered one is registered (an
    // unregistered parser makes the port drop-all); mismatching parsers before
    // that NACK the whole proxylib update (PolicySet::px_nack);
    // HaveL7Rules = some rule has parsed L7 rules.
    bool px_installed = true;
    bool px_have_l7 = false;
};

struct NetworkPolicy {
    std::string name;
    uint64_t id = 0;
    std::vector<PortPolicy> ingress, egress;
    // exact-port entry then port-0 entry (envoy/cilium_network_policy.h:169-192)
    void Lookup(bool ingress, uint32_t port, const PortPolicy **exact, const PortPolicy **wild) const;
};

struct PolicySet {
    std::vector<NetworkPolicy> policies;
    std::map<std::string, int> by_name;
    int nrules = 0;  // global rule ids are 0..nrules-1 in document order
    // Non-empty: the proxylib view NACKs this version (its ParseError panic,
    // recovered in Instance.PolicyUpdate, proxylib/proxylib/instance.go:168-176):
    // "Mismatching L7 types on the same port" (policymap.go:135-143).  Envoy's
    // NPDS accepts the same version (cilium_network_policy.h has no such check),
    // so only the proxylib entry points reject it.
    std::string px_nack;
};

bool LoadPolicySet(const char *json, size_t n, PolicySet *out, std::string *err);
namespace json { struct Value; }
// The same from a parsed tree ({"policies": [...]} or a bare list): the JSON
// path and the NPDS protobuf path (npds_proto.h) both end here.
bool LoadPolicySetTree(const json::Value &root, PolicySet *out, std::string *err);

}  // namespace l7
