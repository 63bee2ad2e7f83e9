"""Independent NPDS encoder for tests: the cilium.NetworkPolicy messages of
envoy/cilium/npds.proto:31-182 (plus the Envoy HeaderMatcher / Int64Range /
DiscoveryResponse / Any they use, field numbers from the reference's generated
Go code: pkg/envoy/envoy/api/v2/route/route.pb.go:3170-3300,
pkg/envoy/envoy/type/range.pb.go:28-30, pkg/envoy/envoy/api/v2/discovery.pb.go:
136-166) declared as descriptors for the Python protobuf runtime, so fixtures
are encoded by Google's serializer, not by the product's decoder's author."""
from google.protobuf import descriptor_pb2, descriptor_pool, json_format, message_factory

F = descriptor_pb2.FieldDescriptorProto
OPT, REP = F.LABEL_OPTIONAL, F.LABEL_REPEATED


def _msg(fd, name, fields, oneofs=(), nested=()):
    m = fd.message_type.add(name=name)
    for o in oneofs:
        m.oneof_decl.add(name=o)
    for n in nested:
        m.nested_type.add().CopyFrom(n)
    for f in fields:
        num, fname, typ, label = f[:4]
        x = m.field.add(name=fname, number=num, type=typ, label=label)
        if len(f) > 4 and f[4]:
            x.type_name = f[4]
        if len(f) > 5 and f[5] is not None:
            x.oneof_index = f[5]
    return m


def _pool():
    pool = descriptor_pool.DescriptorPool()
    fd = descriptor_pb2.FileDescriptorProto(name="npds_test.proto", package="cilium", syntax="proto3")
    T = F
    _msg(fd, "BoolValue", [(1, "value", T.TYPE_BOOL, OPT)])
    _msg(fd, "Int64Range", [(1, "start", T.TYPE_INT64, OPT), (2, "end", T.TYPE_INT64, OPT)])
    _msg(fd, "HeaderMatcher", [
        (1, "name", T.TYPE_STRING, OPT), (4, "exact_match", T.TYPE_STRING, OPT, None, 0),
        (5, "regex_match", T.TYPE_STRING, OPT, None, 0), (6, "range_match", T.TYPE_MESSAGE, OPT, ".cilium.Int64Range", 0),
        (7, "present_match", T.TYPE_BOOL, OPT, None, 0), (9, "prefix_match", T.TYPE_STRING, OPT, None, 0),
        (10, "suffix_match", T.TYPE_STRING, OPT, None, 0), (8, "invert_match", T.TYPE_BOOL, OPT),
        # deprecated in the Envoy C++ route.proto, still used by envoy/cilium_integration_test.cc:779-797
        (2, "value", T.TYPE_STRING, OPT), (3, "regex", T.TYPE_MESSAGE, OPT, ".cilium.BoolValue")],
        oneofs=["header_match_specifier"])
    _msg(fd, "HttpNetworkPolicyRule", [(1, "headers", T.TYPE_MESSAGE, REP, ".cilium.HeaderMatcher")])
    _msg(fd, "HttpNetworkPolicyRules", [(1, "http_rules", T.TYPE_MESSAGE, REP, ".cilium.HttpNetworkPolicyRule")])
    _msg(fd, "KafkaNetworkPolicyRule", [(1, "api_key", T.TYPE_INT32, OPT), (2, "api_version", T.TYPE_INT32, OPT),
                                        (3, "topic", T.TYPE_STRING, OPT), (4, "client_id", T.TYPE_STRING, OPT)])
    _msg(fd, "KafkaNetworkPolicyRules", [(1, "kafka_rules", T.TYPE_MESSAGE, REP, ".cilium.KafkaNetworkPolicyRule")])
    entry = descriptor_pb2.DescriptorProto(name="RuleEntry", options=descriptor_pb2.MessageOptions(map_entry=True))
    entry.field.add(name="key", number=1, type=T.TYPE_STRING, label=OPT)
    entry.field.add(name="value", number=2, type=T.TYPE_STRING, label=OPT)
    _msg(fd, "L7NetworkPolicyRule", [(1, "rule", T.TYPE_MESSAGE, REP, ".cilium.L7NetworkPolicyRule.RuleEntry")],
         nested=[entry])
    _msg(fd, "L7NetworkPolicyRules", [(1, "l7_rules", T.TYPE_MESSAGE, REP, ".cilium.L7NetworkPolicyRule")])
    _msg(fd, "PortNetworkPolicyRule", [
        (1, "remote_policies", T.TYPE_UINT64, REP), (2, "l7_proto", T.TYPE_STRING, OPT),
        (100, "http_rules", T.TYPE_MESSAGE, OPT, ".cilium.HttpNetworkPolicyRules", 0),
        (101, "kafka_rules", T.TYPE_MESSAGE, OPT, ".cilium.KafkaNetworkPolicyRules", 0),
        (102, "l7_rules", T.TYPE_MESSAGE, OPT, ".cilium.L7NetworkPolicyRules", 0)], oneofs=["l7"])
    _msg(fd, "PortNetworkPolicy", [(1, "port", T.TYPE_UINT32, OPT), (2, "protocol", T.TYPE_INT32, OPT),
                                   (3, "rules", T.TYPE_MESSAGE, REP, ".cilium.PortNetworkPolicyRule")])
    _msg(fd, "NetworkPolicy", [(1, "name", T.TYPE_STRING, OPT), (2, "policy", T.TYPE_UINT64, OPT),
                               (3, "ingress_per_port_policies", T.TYPE_MESSAGE, REP, ".cilium.PortNetworkPolicy"),
                               (4, "egress_per_port_policies", T.TYPE_MESSAGE, REP, ".cilium.PortNetworkPolicy")])
    _msg(fd, "Any", [(1, "type_url", T.TYPE_STRING, OPT), (2, "value", T.TYPE_BYTES, OPT)])
    _msg(fd, "DiscoveryResponse", [(1, "version_info", T.TYPE_STRING, OPT), (2, "resources", T.TYPE_MESSAGE, REP, ".cilium.Any"),
                                   (4, "type_url", T.TYPE_STRING, OPT), (5, "nonce", T.TYPE_STRING, OPT)])
    # cilium.LogEntry (pkg/envoy/cilium/accesslog.pb.go:79-400): the access-log records
    _msg(fd, "KeyValue", [(1, "key", T.TYPE_STRING, OPT), (2, "value", T.TYPE_STRING, OPT)])
    _msg(fd, "HttpLogEntry", [(1, "http_protocol", T.TYPE_INT32, OPT), (2, "scheme", T.TYPE_STRING, OPT),
                              (3, "host", T.TYPE_STRING, OPT), (4, "path", T.TYPE_STRING, OPT),
                              (5, "method", T.TYPE_STRING, OPT), (6, "headers", T.TYPE_MESSAGE, REP, ".cilium.KeyValue"),
                              (7, "status", T.TYPE_UINT32, OPT)])
    fentry = descriptor_pb2.DescriptorProto(name="FieldsEntry", options=descriptor_pb2.MessageOptions(map_entry=True))
    fentry.field.add(name="key", number=1, type=T.TYPE_STRING, label=OPT)
    fentry.field.add(name="value", number=2, type=T.TYPE_STRING, label=OPT)
    _msg(fd, "L7LogEntry", [(1, "proto", T.TYPE_STRING, OPT), (2, "fields", T.TYPE_MESSAGE, REP, ".cilium.L7LogEntry.FieldsEntry")],
         nested=[fentry])
    _msg(fd, "LogEntry", [
        (1, "timestamp", T.TYPE_UINT64, OPT), (15, "is_ingress", T.TYPE_BOOL, OPT), (3, "entry_type", T.TYPE_INT32, OPT),
        (4, "policy_name", T.TYPE_STRING, OPT), (5, "cilium_rule_ref", T.TYPE_STRING, OPT),
        (6, "source_security_id", T.TYPE_UINT32, OPT), (16, "destination_security_id", T.TYPE_UINT32, OPT),
        (7, "source_address", T.TYPE_STRING, OPT), (8, "destination_address", T.TYPE_STRING, OPT),
        (100, "http", T.TYPE_MESSAGE, OPT, ".cilium.HttpLogEntry", 0),
        (102, "generic_l7", T.TYPE_MESSAGE, OPT, ".cilium.L7LogEntry", 0)], oneofs=["l7"])
    pool.Add(fd)
    return pool


_POOL = _pool()


def cls(name):
    return message_factory.GetMessageClass(_POOL.FindMessageTypeByName("cilium." + name))


def _matcher(m):
    m = dict(m)
    if isinstance(m.get("regex"), bool):
        m["regex"] = {"value": m["regex"]}
    return m


def _normalize(np_json):
    """Our JSON policy shape -> the NPDS proto field layout (protocol enum as
    its number; L7 rule maps wrapped as in the proto)."""
    d = dict(np_json)
    for k in ("ingress_per_port_policies", "egress_per_port_policies"):
        ports = []
        for p in d.get(k, []):
            p = dict(p)
            if isinstance(p.get("protocol"), str):
                p["protocol"] = 1 if p["protocol"] == "UDP" else 0
            rules = []
            for r in p.get("rules", []):
                r = dict(r)
                if "http_rules" in r:
                    r["http_rules"] = {"http_rules": [dict(h, headers=[_matcher(m) for m in h.get("headers", [])])
                                                      for h in r["http_rules"]["http_rules"]]}
                if "l7_rules" in r:
                    r["l7_rules"] = {"l7_rules": [{"rule": x["rule"]} for x in r["l7_rules"]["l7_rules"]]}
                rules.append(r)
            p["rules"] = rules
            ports.append(p)
        d[k] = ports
    return d


def network_policy(np_json):
    return json_format.ParseDict(_normalize(np_json), cls("NetworkPolicy")())


def discovery_response(policy_set, version="1"):
    resp = cls("DiscoveryResponse")(version_info=version, type_url="type.googleapis.com/cilium.NetworkPolicy")
    for p in policy_set["policies"]:
        a = resp.resources.add()
        a.type_url = "type.googleapis.com/cilium.NetworkPolicy"
        a.value = network_policy(p).SerializeToString()
    return resp.SerializeToString()
