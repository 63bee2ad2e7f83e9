// Policy ingestion and validation (product code).  Rejects exactly what the
// reference rejects, so a policy that would be NACKed there fails here:
//   * duplicate TCP port per direction  envoy/cilium_network_policy.h:158-160
//   * HTTP regex must parse (Go syntax) pkg/policy/api/http.go:66-84
//   * PortRuleKafka.Sanitize            pkg/policy/api/rule_validation.go:232-275
//   * one L7 oneof per rule             envoy/cilium/npds.proto:91-106
//   * unique remote_policies            npds.proto:77 (validate.rules)
#include "policy.h"

#include "../engine/mc_groups.h"

#include <algorithm>
#include <cctype>
#include <cstring>

#include "json.h"
#include "../kernels/cass_parse.h"

namespace l7 {

bool PortRule::RemoteOk(uint64_t id) const {
    if (remotes.empty()) return true;
    return std::binary_search(remotes.begin(), remotes.end(), id);
}

bool ProxylibParserRegistered(const std::string &name) {
    // the reference's libcilium links cassandra, memcached, r2d2 and the test
    // parsers (proxylib/proxylib.go:24-29), whose init()s register the rule
    // parsers "cassandra", "memcache", "r2d2" and "test.headerparser"; the
    // HTTP / Kafka oneof parsers are this library's proxylib "http" / "kafka"
    return name.empty() || name == "memcache" || name == "r2d2" || name == "cassandra" ||
           name == "test.headerparser" || name == "PortNetworkPolicyRule_HttpRules" ||
           name == "PortNetworkPolicyRule_KafkaRules";
}

std::string PortRule::ParserName() const {
    if (!l7proto.empty()) return l7proto;
    switch (type) {
        case Http: return "PortNetworkPolicyRule_HttpRules";
        case Kafka: return "PortNetworkPolicyRule_KafkaRules";
        case L7: return "PortNetworkPolicyRule_L7Rules";
        default: return "";
    }
}

void NetworkPolicy::Lookup(bool in, uint32_t port, const PortPolicy **exact, const PortPolicy **wild) const {
    const auto &v = in ? ingress : egress;
    *exact = *wild = nullptr;
    for (auto &p : v) {
        if (!p.tcp) continue;
        if (p.port == port) *exact = &p;
        if (p.port == 0 && port != 0) *wild = &p;
    }
}

namespace {

using json::Value;

struct Loader {
    std::string err;
    int next_id = 0;
    bool mc_stop = false;  // an earlier rule of this port has an unregistered parser
    std::string px_nack;   // first proxylib ParseError of this version (PolicySet::px_nack)
    bool fail(const std::string &m) { if (err.empty()) err = m; return false; }

    static const Value *list(const Value *v, const char *inner) {
        if (!v) return nullptr;
        if (v->isArr()) return v;
        if (v->isObj()) { auto *a = v->get(inner); if (a && a->isArr()) return a; }
        return nullptr;
    }
    static bool str(const Value &o, const char *k, std::string *s) {
        auto *v = o.get(k);
        if (!v || !v->isStr()) return false;
        *s = v->str;
        return true;
    }

    bool matcher(const Value &j, HeaderMatcher *h) {
        if (!str(j, "name", &h->name)) return fail("header matcher without name");
        for (auto &c : h->name) c = (char)std::tolower((unsigned char)c);
        auto *inv = j.get("invert_match");
        h->invert = inv && inv->type == Value::Bool && inv->b;
        const Value *v;
        if (str(j, "exact_match", &h->value)) h->type = HM::Exact;
        else if (str(j, "regex_match", &h->value)) h->type = HM::Regex;
        else if (str(j, "prefix_match", &h->value)) h->type = HM::Prefix;
        else if (str(j, "suffix_match", &h->value)) h->type = HM::Suffix;
        else if ((v = j.get("present_match")) && v->type == Value::Bool) h->type = HM::Present;
        else if ((v = j.get("range_match")) && v->isObj()) {
            h->type = HM::Range;
            auto *a = v->get("start"), *b = v->get("end");
            h->rstart = a ? a->inum : 0;
            h->rend = b ? b->inum : 0;
        } else if (str(j, "value", &h->value)) {  // deprecated value + regex flag
            auto *r = j.get("regex");
            h->type = (r && r->type == Value::Bool && r->b) ? HM::Regex : HM::Exact;
        } else {
            h->type = HM::Exact;  // empty ExactMatch == presence
        }
        if (h->type == HM::Regex) {
            std::string e;
            auto ast = re::Parse(h->value, &e);
            if (!ast) return fail(e);
            h->ast = std::shared_ptr<re::Node>(std::move(ast));
        }
        return true;
    }

    static bool ieq(const std::string &a, const char *b) {
        size_t n = strlen(b);
        if (a.size() != n) return false;
        for (size_t i = 0; i < n; i++) if (std::tolower((unsigned char)a[i]) != b[i]) return false;
        return true;
    }
    static bool parseInt16(const std::string &s, int16_t *out) {  // strconv.ParseInt(s, 10, 16)
        size_t i = 0;
        bool neg = false;
        if (s.empty()) return false;
        if (s[0] == '+' || s[0] == '-') { neg = s[0] == '-'; i = 1; }
        if (i >= s.size()) return false;
        long v = 0;
        for (; i < s.size(); i++) {
            if (s[i] < '0' || s[i] > '9') return false;
            v = v * 10 + (s[i] - '0');
            if (v > 40000) return false;
        }
        if (neg) v = -v;
        if (v < -32768 || v > 32767) return false;
        *out = (int16_t)v;
        return true;
    }

    bool kafka(const Value &j, KafkaRule *k) {
        static const char *kKeys[] = {
            "produce", "fetch", "offsets", "metadata", "leaderandisr", "stopreplica", "updatemetadata",
            "controlledshutdown", "offsetcommit", "offsetfetch", "findcoordinator", "joingroup", "heartbeat",
            "leavegroup", "syncgroup", "describegroups", "listgroups", "saslhandshake", "apiversions",
            "createtopics", "deletetopics", "deleterecords", "initproducerid", "offsetforleaderepoch",
            "addpartitionstotxn", "addoffsetstotxn", "endtxn", "writetxnmarkers", "txnoffsetcommit",
            "describeacls", "createacls", "deleteacls", "describeconfigs", "alterconfigs"};
        std::string role, key, ver, s;
        str(j, "role", &role);
        str(j, "apiKey", &key);
        if (!role.empty() && !key.empty())
            return fail("Cannot set both Role:\"" + role + "\" and APIKey :\"" + key + "\" together");
        if (!key.empty()) {
            int found = -1;
            for (int i = 0; i < (int)(sizeof kKeys / sizeof kKeys[0]); i++) if (ieq(key, kKeys[i])) found = i;
            if (found < 0) return fail("invalid Kafka APIKey :\"" + key + "\"");
            k->any_key = false;
            k->keymask |= 1ull << found;
        }
        if (!role.empty()) {
            k->any_key = false;
            if (ieq(role, "produce")) k->keymask = (1ull << 0) | (1ull << 3) | (1ull << 18);
            else if (ieq(role, "consume")) {
                for (int x : {1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18}) k->keymask |= 1ull << x;
            } else return fail("invalid Kafka APIRole :\"" + role + "\"");
        }
        if (str(j, "apiVersion", &ver) && !ver.empty()) {
            if (!parseInt16(ver, &k->version)) return fail("invalid Kafka APIVersion :\"" + ver + "\"");
            k->has_version = true;
        }
        if (str(j, "topic", &s) && !s.empty()) {
            if (s.size() > 255) return fail("kafka topic exceeds maximum len of 255");
            for (unsigned char c : s)  // KafkaTopicValidChar ^[a-zA-Z0-9\\._\\-]+$ (admits '\')
                if (!(std::isalnum(c) || c == '\\' || c == '.' || c == '_' || c == '-')) return fail("invalid Kafka Topic name \"" + s + "\"");
            k->topic = s;
        }
        if ((str(j, "clientID", &s) || str(j, "client_id", &s)) && !s.empty()) k->client = s;
        const Value *v;
        if ((v = j.get("api_key")) && v->type == Value::Num && v->inum >= 0) {  // NPDS KafkaNetworkPolicyRule form
            if (v->inum > 63) return fail("kafka api_key out of range");
            k->any_key = false;
            k->keymask = 1ull << v->inum;
        }
        if ((v = j.get("api_version")) && v->type == Value::Num && v->inum >= 0) { k->has_version = true; k->version = (int16_t)v->inum; }
        return true;
    }

    bool rule(const Value &j, PortRule *r) {
        if (auto *rp = j.get("remote_policies"); rp && rp->isArr()) {
            for (auto &x : rp->arr) r->remotes.push_back((uint64_t)x.inum);
            std::vector<uint64_t> s = r->remotes;
            std::sort(s.begin(), s.end());
            if (std::adjacent_find(s.begin(), s.end()) != s.end()) return fail("remote_policies must be unique");
            r->remotes = s;
        }
        str(j, "l7_proto", &r->l7proto);
        auto *h = list(j.get("http_rules"), "http_rules");
        auto *kf = list(j.get("kafka_rules"), "kafka_rules");
        auto *l = list(j.get("l7_rules"), "l7_rules");
        if ((h != nullptr) + (kf != nullptr) + (l != nullptr) > 1) return fail("more than one L7 rule type in a rule");
        if (h) {
            r->type = PortRule::Http;
            for (auto &hr : h->arr) {
                HttpRule x;
                x.id = next_id++;
                if (auto *hs = hr.get("headers"); hs && hs->isArr())
                    for (auto &m : hs->arr) { x.m.emplace_back(); if (!matcher(m, &x.m.back())) return false; }
                r->http.push_back(std::move(x));
            }
        } else if (kf) {
            r->type = PortRule::Kafka;
            for (auto &kr : kf->arr) {
                KafkaRule x;
                if (!kafka(kr, &x)) return false;
                x.id = next_id++;
                r->kafka.push_back(std::move(x));
            }
        } else if (l) {
            r->type = PortRule::L7;
            for (auto &lr : l->arr) {
                L7Rule x;
                x.id = next_id++;
                const Value *m = lr.get("rule");
                if (!m) m = &lr;
                if (m->isObj())
                    for (auto &kv : m->obj) {
                        if (kv.second.isStr()) x.kv.emplace_back(kv.first, kv.second.str);
                        else if ((r->l7proto == "memcache" || r->l7proto == "r2d2" || r->l7proto == "cassandra") && !mc_stop)
                            return fail("NPDS: " + r->l7proto + " rule value is not a string");
                    }
                r->l7.push_back(std::move(x));
            }
            if (r->l7proto == "memcache" && !mc_stop)
                for (auto &x : r->l7) {
                    r->mc.emplace_back();
                    if (!memcache(x, &r->mc.back())) return false;
                }
            if (r->l7proto == "test.headerparser") r->other_l7 = r->l7.size();
            if (r->l7proto == "cassandra" && !mc_stop)
                for (auto &x : r->l7) {
                    r->cass.emplace_back();
                    if (!cassandra(x, &r->cass.back())) return false;
                }
            if (r->l7proto == "r2d2" && !mc_stop)
                for (auto &x : r->l7) {
                    r->r2.emplace_back();
                    if (!r2d2(x, &r->r2.back())) return false;
                }
        }
        return true;
    }

    // memcache.L7RuleParser (proxylib/memcached/parser.go:114-148)
    bool memcache(const L7Rule &x, McRule *m) {
        m->id = x.id;
        bool found = false;
        for (auto &kv : x.kv) {
            const std::string &k = kv.first, &v = kv.second;
            if (k == "command") { m->group = McGroupIndex(v); found = m->group >= 0; }
            else if (k == "keyExact") m->key_exact = v;
            else if (k == "keyPrefix") m->key_prefix = v;
            else if (k == "keyRegex") {
                std::string e;
                auto ast = re::Parse(v, &e);
                if (!ast) return fail(e);
                m->key_re = std::shared_ptr<re::Node>(std::move(ast));
                m->key_re_src = v;
            } else return fail("NPDS: Unsupported key: " + k);
        }
        if (!found) {
            if (!m->key_exact.empty() || !m->key_prefix.empty() || m->key_re)
                return fail("NPDS: command not specified but key was provided");
            m->group = -1;
            m->empty = true;
        }
        return true;
    }

    // r2d2.R2d2RuleParser (proxylib/r2d2/r2d2parser.go:69-107); its panics
    // (ParseError, regexp.MustCompile) NACK the policy
    bool r2d2(const L7Rule &x, R2Rule *m) {
        m->id = x.id;
        std::string cmd;
        for (auto &kv : x.kv) {
            const std::string &k = kv.first, &v = kv.second;
            if (k == "cmd") cmd = v;
            else if (k == "file") {
                if (v.empty()) continue;
                std::string e;
                auto ast = re::Parse(v, &e);
                if (!ast) return fail("regexp: Compile(`" + v + "`): " + e);  // regexp.MustCompile's panic
                m->file_re = std::shared_ptr<re::Node>(std::move(ast));
                m->file_src = v;
            } else {
                return fail("NPDS: Unsupported key: " + k);
            }
        }
        if (!cmd.empty() && cmd != "READ" && cmd != "WRITE" && cmd != "HALT" && cmd != "RESET")
            return fail("NPDS: Unable to parse L7 r2d2 rule with invalid cmd: '" + cmd + "'");
        if (m->file_re && !(cmd.empty() || cmd == "READ" || cmd == "WRITE"))
            return fail("NPDS: Unable to parse L7 r2d2 rule, cmd '" + cmd + "' is not compatible with 'file'");
        m->cmd = cmd.empty() ? -1 : cmd == "READ" ? R2_READ : cmd == "WRITE" ? R2_WRITE : cmd == "HALT" ? R2_HALT : R2_RESET;
        return true;
    }

    // cassandra.CassandraRuleParser (proxylib/cassandra/cassandraparser.go:99-134);
    // its ParseError / regexp.MustCompile panics NACK the policy
    bool cassandra(const L7Rule &x, CassRule *m) {
        m->id = x.id;
        std::string action;
        bool has_action = false;
        for (auto &kv : x.kv) {
            const std::string &k = kv.first, &v = kv.second;
            if (k == "query_action") {
                action = v;
                has_action = !v.empty();
            } else if (k == "query_table") {
                if (v.empty()) continue;
                std::string e;
                auto ast = re::Parse(v, &e);
                if (!ast) return fail("regexp: Compile(`" + v + "`): " + e);
                m->table_re = std::shared_ptr<re::Node>(std::move(ast));
                m->table_src = v;
            } else {
                return fail("NPDS: Unsupported key: " + k);
            }
        }
        if (has_action) {
            m->action = -1;
            for (int a = 0; a < kCassActions; a++)
                if (action == CassActionName(a)) m->action = a;
            if (m->action < 0)
                return fail("NPDS: Unable to parse L7 cassandra rule with invalid query_action: '" + action + "'");
            if (m->action >= kCassTableActions && m->table_re)
                return fail("NPDS: query_action '" + action + "' is not compatible with a query_table match");
        }
        return true;
    }

    bool ports(const Value *arr, std::vector<PortPolicy> *out) {
        if (!arr || !arr->isArr()) return true;
        for (auto &pj : arr->arr) {
            PortPolicy p;
            auto *pv = pj.get("port");
            int64_t port = pv ? pv->inum : 0;
            if (port < 0 || port > 65535) return fail("port out of range");
            p.port = (uint32_t)port;
            if (auto *pr = pj.get("protocol")) {
                if (pr->isStr() && pr->str == "UDP") p.tcp = false;
                if (pr->type == Value::Num && pr->inum != 0) p.tcp = false;
            }
            mc_stop = false;
            std::string first_parser;
            if (auto *rs = pj.get("rules"); rs && rs->isArr())
                for (auto &rj : rs->arr) {
                    p.rules.emplace_back();
                    PortRule &r = p.rules.back();
                    if (!rule(rj, &r)) return false;
                    if (r.type == PortRule::Http) p.has_http = true;
                    std::string pn = r.ParserName();
                    // newPortNetworkPolicyRules (policymap.go:113-148), rule by rule:
                    // an unregistered parser returns the port as drop-all at once
                    // (later rules are never parsed, :128-134); a registered one whose
                    // name differs from the port's first is a ParseError panic that
                    // NACKs the whole proxylib update (:135-143).  UDP ports are never
                    // parsed by proxylib (:206-209).
                    if (!mc_stop) {
                        if (!ProxylibParserRegistered(pn)) {
                            mc_stop = true;
                            p.px_installed = false;
                        } else if (!pn.empty()) {
                            if (first_parser.empty()) first_parser = pn;
                            else if (pn != first_parser && p.tcp && px_nack.empty())
                                px_nack = "NPDS: Mismatching L7 types on the same port";
                        }
                    }
                    if (!mc_stop && r.NumL7() > 0) p.px_have_l7 = true;
                }
            if (p.tcp)
                for (auto &q : *out) if (q.tcp && q.port == p.port) return fail("PortNetworkPolicy: Duplicate port number");
            out->push_back(std::move(p));
        }
        return true;
    }
};

}  // namespace

bool LoadPolicySet(const char *js, size_t n, PolicySet *out, std::string *err) {
    json::Value root;
    if (!json::Parse(js, n, &root, err)) return false;
    return LoadPolicySetTree(root, out, err);
}

bool LoadPolicySetTree(const json::Value &root, PolicySet *out, std::string *err) {
    const json::Value *arr = root.isObj() ? root.get("policies") : &root;
    if (!arr || !arr->isArr()) { if (err) *err = "expected a list of policies"; return false; }
    Loader L;
    PolicySet ps;
    for (auto &pj : arr->arr) {
        NetworkPolicy np;
        Loader::str(pj, "name", &np.name);
        if (auto *id = pj.get("policy")) np.id = (uint64_t)id->inum;
        if (!L.ports(pj.get("ingress_per_port_policies"), &np.ingress) ||
            !L.ports(pj.get("egress_per_port_policies"), &np.egress)) {
            if (err) *err = L.err;
            return false;
        }
        ps.by_name.emplace(np.name, (int)ps.policies.size());
        ps.policies.push_back(std::move(np));
    }
    ps.nrules = L.next_id;
    ps.px_nack = L.px_nack;
    *out = std::move(ps);
    return true;
}

}  // namespace l7
