// NPDS protobuf ingestion (product code): a hand-written proto3 wire-format
// decoder for the cilium.NetworkPolicy resources of an NPDS
// envoy.api.v2.DiscoveryResponse, lowered onto the same policy tree the JSON
// path reads (policy.cc), so both deliveries compile to identical tables.
//
//   envoy/cilium/npds.proto:31-182            NetworkPolicy .. L7NetworkPolicyRule
//   pkg/envoy/envoy/api/v2/discovery.pb.go:136-166   DiscoveryResponse (resources = 2)
//   pkg/envoy/envoy/api/v2/route/route.pb.go:3170-3300  HeaderMatcher fields (+ the
//                                             deprecated value = 2 / regex = 3 the Envoy side still reads)
//   pkg/envoy/envoy/type/range.pb.go:28-30    Int64Range
//   proxylib/proxylib/instance.go:168-219     policy update: all resources or none
//
// proto3 rules kept: unknown fields are skipped; a scalar repeated field may
// arrive packed or not; the last member of a oneof wins; absent scalars read
// as their zero value (so an absent KafkaNetworkPolicyRule.api_key is 0, i.e.
// produce, exactly as the reference's generated code reads it).
#include "npds_proto.h"

#include <cstring>

namespace l7 {

namespace {

using json::Value;

struct Reader {
    const uint8_t *p, *e;
    bool ok = true;
    bool done() const { return p >= e || !ok; }
    uint64_t varint() {
        uint64_t v = 0;
        for (int s = 0; s < 70; s += 7) {
            if (p >= e) { ok = false; return 0; }
            const uint8_t b = *p++;
            v |= (uint64_t)(b & 0x7F) << s;
            if (!(b & 0x80)) return v;
        }
        ok = false;  // more than 10 bytes
        return 0;
    }
    // field key -> (number, wire type)
    bool key(uint32_t *field, uint32_t *wt) {
        const uint64_t k = varint();
        *field = (uint32_t)(k >> 3);
        *wt = (uint32_t)(k & 7);
        if (ok && *field == 0) ok = false;
        return ok;
    }
    bool bytes(const uint8_t **b, size_t *n) {
        const uint64_t len = varint();
        if (!ok || len > (uint64_t)(e - p)) { ok = false; return false; }
        *b = p;
        *n = (size_t)len;
        p += len;
        return true;
    }
    void skip(uint32_t wt) {
        const uint8_t *b;
        size_t n;
        switch (wt) {
        case 0: varint(); break;
        case 1: if (e - p < 8) ok = false; else p += 8; break;
        case 2: bytes(&b, &n); break;
        case 5: if (e - p < 4) ok = false; else p += 4; break;
        default: ok = false; break;  // groups are not proto3
        }
    }
};

Value Str(const uint8_t *b, size_t n) {
    Value v;
    v.type = Value::Str;
    v.str.assign((const char *)b, n);
    return v;
}
Value Num(int64_t x) {
    Value v;
    v.type = Value::Num;
    v.inum = x;
    v.num = (double)x;
    return v;
}
Value Bool(bool x) {
    Value v;
    v.type = Value::Bool;
    v.b = x;
    return v;
}
Value Obj() {
    Value v;
    v.type = Value::Obj;
    return v;
}
Value Arr() {
    Value v;
    v.type = Value::Arr;
    return v;
}
// set (replace) member k of object o
void Set(Value &o, const char *k, Value v) {
    for (auto &kv : o.obj)
        if (kv.first == k) { kv.second = std::move(v); return; }
    o.obj.emplace_back(k, std::move(v));
}
void Erase(Value &o, const char *k) {
    for (size_t i = 0; i < o.obj.size(); i++)
        if (o.obj[i].first == k) { o.obj.erase(o.obj.begin() + i); return; }
}
Value &Member(Value &o, const char *k, Value init) {
    for (auto &kv : o.obj)
        if (kv.first == k) return kv.second;
    o.obj.emplace_back(k, std::move(init));
    return o.obj.back().second;
}

struct Decoder {
    std::string err;
    bool fail(const std::string &m) { if (err.empty()) err = m; return false; }

    // a length-delimited field as a sub-reader
    bool sub(Reader &r, uint32_t wt, Reader *s, const char *what) {
        const uint8_t *b;
        size_t n;
        if (wt != 2 || !r.bytes(&b, &n)) return fail(std::string("NPDS: malformed ") + what);
        *s = Reader{b, b + n};
        return true;
    }
    bool string(Reader &r, uint32_t wt, Value *out, const char *what) {
        const uint8_t *b;
        size_t n;
        if (wt != 2 || !r.bytes(&b, &n)) return fail(std::string("NPDS: malformed ") + what);
        *out = Str(b, n);
        return true;
    }
    bool scalar(Reader &r, uint32_t wt, uint64_t *v, const char *what) {
        if (wt != 0) return fail(std::string("NPDS: malformed ") + what);
        *v = r.varint();
        return r.ok || fail(std::string("NPDS: malformed ") + what);
    }

    // envoy.type.Int64Range
    bool range(Reader r, Value *out) {
        *out = Obj();
        Set(*out, "start", Num(0));
        Set(*out, "end", Num(0));
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            uint64_t v;
            if (f == 1 || f == 2) {
                if (!scalar(r, wt, &v, "Int64Range")) return false;
                Set(*out, f == 1 ? "start" : "end", Num((int64_t)v));
            } else {
                r.skip(wt);
            }
        }
        return r.ok || fail("NPDS: malformed Int64Range");
    }

    // envoy.api.v2.route.HeaderMatcher
    bool matcher(Reader r, Value *out) {
        *out = Obj();
        const char *spec[] = {"exact_match", "regex_match", "range_match", "present_match", "prefix_match", "suffix_match"};
        auto clear_spec = [&] { for (const char *k : spec) Erase(*out, k); };
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            Value v;
            uint64_t x;
            switch (f) {
            case 1: if (!string(r, wt, &v, "HeaderMatcher.name")) return false; Set(*out, "name", v); break;
            case 4: if (!string(r, wt, &v, "HeaderMatcher")) return false; clear_spec(); Set(*out, "exact_match", v); break;
            case 5: if (!string(r, wt, &v, "HeaderMatcher")) return false; clear_spec(); Set(*out, "regex_match", v); break;
            case 6: {
                Reader s{nullptr, nullptr};
                if (!sub(r, wt, &s, "HeaderMatcher.range_match") || !range(s, &v)) return false;
                clear_spec();
                Set(*out, "range_match", v);
                break;
            }
            case 7: if (!scalar(r, wt, &x, "HeaderMatcher")) return false; clear_spec(); Set(*out, "present_match", Bool(x != 0)); break;
            case 8: if (!scalar(r, wt, &x, "HeaderMatcher")) return false; Set(*out, "invert_match", Bool(x != 0)); break;
            // the deprecated value / regex pair of the Envoy C++ side's route.proto
            // (what envoy/cilium_integration_test.cc:779-797 still writes)
            case 2: if (!string(r, wt, &v, "HeaderMatcher.value")) return false; Set(*out, "value", v); break;
            case 3: {  // google.protobuf.BoolValue
                Reader s{nullptr, nullptr};
                if (!sub(r, wt, &s, "HeaderMatcher.regex")) return false;
                bool rx = false;
                uint32_t g, wt2;
                while (!s.done() && s.key(&g, &wt2)) {
                    if (g == 1) { if (!scalar(s, wt2, &x, "BoolValue")) return false; rx = x != 0; }
                    else s.skip(wt2);
                }
                if (!s.ok) return fail("NPDS: malformed HeaderMatcher.regex");
                Set(*out, "regex", Bool(rx));
                break;
            }
            case 9: if (!string(r, wt, &v, "HeaderMatcher")) return false; clear_spec(); Set(*out, "prefix_match", v); break;
            case 10: if (!string(r, wt, &v, "HeaderMatcher")) return false; clear_spec(); Set(*out, "suffix_match", v); break;
            default: r.skip(wt); break;
            }
        }
        // an absent name reads as "" (proto3); the JSON loader wants the key
        if (!out->get("name")) Set(*out, "name", Str(nullptr, 0));
        // no specifier: proto3's unset oneof = exact_match "" (presence) in the JSON loader
        return r.ok || fail("NPDS: malformed HeaderMatcher");
    }

    // repeated message field `inner` (field 1) of a wrapper message, appended to arr
    template <class F>
    bool wrapped_list(Reader r, Value *arr, const char *what, F item) {
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            if (f != 1) { r.skip(wt); continue; }
            Reader s{nullptr, nullptr};
            if (!sub(r, wt, &s, what)) return false;
            Value v;
            if (!item(s, &v)) return false;
            arr->arr.push_back(std::move(v));
        }
        return r.ok || fail(std::string("NPDS: malformed ") + what);
    }

    bool http_rule(Reader r, Value *out) {  // HttpNetworkPolicyRule
        *out = Obj();
        Value hs = Arr();
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            if (f != 1) { r.skip(wt); continue; }
            Reader s{nullptr, nullptr};
            Value m;
            if (!sub(r, wt, &s, "HttpNetworkPolicyRule") || !matcher(s, &m)) return false;
            hs.arr.push_back(std::move(m));
        }
        Set(*out, "headers", std::move(hs));
        return r.ok || fail("NPDS: malformed HttpNetworkPolicyRule");
    }

    bool kafka_rule(Reader r, Value *out) {  // KafkaNetworkPolicyRule (absent ints are 0)
        *out = Obj();
        Set(*out, "api_key", Num(0));
        Set(*out, "api_version", Num(0));
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            Value v;
            uint64_t x;
            switch (f) {
            case 1: if (!scalar(r, wt, &x, "KafkaNetworkPolicyRule")) return false; Set(*out, "api_key", Num((int32_t)x)); break;
            case 2: if (!scalar(r, wt, &x, "KafkaNetworkPolicyRule")) return false; Set(*out, "api_version", Num((int32_t)x)); break;
            case 3: if (!string(r, wt, &v, "KafkaNetworkPolicyRule")) return false; Set(*out, "topic", v); break;
            case 4: if (!string(r, wt, &v, "KafkaNetworkPolicyRule")) return false; Set(*out, "client_id", v); break;
            default: r.skip(wt); break;
            }
        }
        return r.ok || fail("NPDS: malformed KafkaNetworkPolicyRule");
    }

    bool l7_rule(Reader r, Value *out) {  // L7NetworkPolicyRule: map<string, string> rule = 1
        *out = Obj();
        Value &m = Member(*out, "rule", Obj());
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            if (f != 1) { r.skip(wt); continue; }
            Reader s{nullptr, nullptr};
            if (!sub(r, wt, &s, "L7NetworkPolicyRule")) return false;
            Value k = Str(nullptr, 0), v = Str(nullptr, 0);
            uint32_t g, wt2;
            while (!s.done() && s.key(&g, &wt2)) {
                if (g == 1) { if (!string(s, wt2, &k, "map entry")) return false; }
                else if (g == 2) { if (!string(s, wt2, &v, "map entry")) return false; }
                else s.skip(wt2);
            }
            if (!s.ok) return fail("NPDS: malformed L7NetworkPolicyRule");
            Set(m, k.str.c_str(), std::move(v));  // a repeated key: the last entry wins
        }
        return r.ok || fail("NPDS: malformed L7NetworkPolicyRule");
    }

    bool port_rule(Reader r, Value *out) {  // PortNetworkPolicyRule
        *out = Obj();
        Value remotes = Arr();
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            Value v;
            Reader s{nullptr, nullptr};
            switch (f) {
            case 1:  // repeated uint64, packed or not
                if (wt == 2) {
                    if (!sub(r, wt, &s, "remote_policies")) return false;
                    while (!s.done()) remotes.arr.push_back(Num((int64_t)s.varint()));
                    if (!s.ok) return fail("NPDS: malformed remote_policies");
                } else {
                    uint64_t x;
                    if (!scalar(r, wt, &x, "remote_policies")) return false;
                    remotes.arr.push_back(Num((int64_t)x));
                }
                break;
            case 2: if (!string(r, wt, &v, "l7_proto")) return false; Set(*out, "l7_proto", v); break;
            case 100: case 101: case 102: {
                const char *name = f == 100 ? "http_rules" : f == 101 ? "kafka_rules" : "l7_rules";
                if (!sub(r, wt, &s, name)) return false;
                Value arr = Arr();
                bool ok = f == 100 ? wrapped_list(s, &arr, name, [&](Reader x, Value *o) { return http_rule(x, o); })
                        : f == 101 ? wrapped_list(s, &arr, name, [&](Reader x, Value *o) { return kafka_rule(x, o); })
                                   : wrapped_list(s, &arr, name, [&](Reader x, Value *o) { return l7_rule(x, o); });
                if (!ok) return false;
                for (const char *k : {"http_rules", "kafka_rules", "l7_rules"}) Erase(*out, k);  // oneof: the last wins
                Set(*out, name, std::move(arr));
                break;
            }
            default: r.skip(wt); break;
            }
        }
        if (!remotes.arr.empty()) Set(*out, "remote_policies", std::move(remotes));
        return r.ok || fail("NPDS: malformed PortNetworkPolicyRule");
    }

    bool port_policy(Reader r, Value *out) {  // PortNetworkPolicy
        *out = Obj();
        Set(*out, "port", Num(0));
        Value rules = Arr();
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            uint64_t x;
            Reader s{nullptr, nullptr};
            Value v;
            switch (f) {
            case 1: if (!scalar(r, wt, &x, "PortNetworkPolicy.port")) return false; Set(*out, "port", Num((int64_t)(uint32_t)x)); break;
            case 2: if (!scalar(r, wt, &x, "PortNetworkPolicy.protocol")) return false; Set(*out, "protocol", Num((int64_t)(int32_t)x)); break;
            case 3:
                if (!sub(r, wt, &s, "PortNetworkPolicyRule") || !port_rule(s, &v)) return false;
                rules.arr.push_back(std::move(v));
                break;
            default: r.skip(wt); break;
            }
        }
        Set(*out, "rules", std::move(rules));
        return r.ok || fail("NPDS: malformed PortNetworkPolicy");
    }

    bool network_policy(Reader r, Value *out) {  // NetworkPolicy
        *out = Obj();
        Set(*out, "name", Str(nullptr, 0));
        Set(*out, "policy", Num(0));
        Value in = Arr(), eg = Arr();
        uint32_t f, wt;
        while (!r.done() && r.key(&f, &wt)) {
            uint64_t x;
            Reader s{nullptr, nullptr};
            Value v;
            switch (f) {
            case 1: if (!string(r, wt, &v, "NetworkPolicy.name")) return false; Set(*out, "name", v); break;
            case 2: if (!scalar(r, wt, &x, "NetworkPolicy.policy")) return false; Set(*out, "policy", Num((int64_t)x)); break;
            case 3: case 4:
                if (!sub(r, wt, &s, "PortNetworkPolicy") || !port_policy(s, &v)) return false;
                (f == 3 ? in : eg).arr.push_back(std::move(v));
                break;
            default: r.skip(wt); break;
            }
        }
        Set(*out, "ingress_per_port_policies", std::move(in));
        Set(*out, "egress_per_port_policies", std::move(eg));
        return r.ok || fail("NPDS: malformed NetworkPolicy");
    }
};

constexpr char kTypeUrl[] = "type.googleapis.com/cilium.NetworkPolicy";

}  // namespace

bool NpdsResponseToTree(const uint8_t *buf, size_t len, json::Value *root, std::string *version, std::string *err) {
    Decoder D;
    Reader r{buf, buf + len};
    *root = Obj();
    Value pols = Arr();
    if (version) version->clear();
    uint32_t f, wt;
    while (!r.done() && r.key(&f, &wt)) {
        Reader s{nullptr, nullptr};
        Value v;
        if (f == 1) {  // version_info
            if (!D.string(r, wt, &v, "DiscoveryResponse.version_info")) break;
            if (version) *version = v.str;
        } else if (f == 2) {  // resources: google.protobuf.Any
            if (!D.sub(r, wt, &s, "DiscoveryResponse.resources")) break;
            std::string url;
            const uint8_t *vb = nullptr;
            size_t vn = 0;
            uint32_t g, wt2;
            while (!s.done() && s.key(&g, &wt2)) {
                if (g == 1) { Value u; if (!D.string(s, wt2, &u, "Any.type_url")) break; url = u.str; }
                else if (g == 2) { if (wt2 != 2 || !s.bytes(&vb, &vn)) { D.fail("NPDS: malformed Any.value"); break; } }
                else s.skip(wt2);
            }
            if (!D.err.empty()) break;
            if (!s.ok) { D.fail("NPDS: malformed Any"); break; }
            if (url != kTypeUrl) { D.fail("NPDS: unexpected resource type \"" + url + "\""); break; }
            Value np;
            if (!D.network_policy(Reader{vb, vb + vn}, &np)) break;
            pols.arr.push_back(std::move(np));
        } else {
            r.skip(wt);
        }
    }
    if (D.err.empty() && !r.ok) D.fail("NPDS: malformed DiscoveryResponse");
    if (!D.err.empty()) {
        if (err) *err = D.err;
        return false;
    }
    Set(*root, "policies", std::move(pols));
    return true;
}

bool LoadPolicySetProto(const uint8_t *buf, size_t len, PolicySet *out, std::string *err) {
    json::Value root;
    if (!NpdsResponseToTree(buf, len, &root, nullptr, err)) return false;
    return LoadPolicySetTree(root, out, err);
}

}  // namespace l7
