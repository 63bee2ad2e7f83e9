"""NPDS protobuf ingestion (l7g_policy_update_proto), host-only engine.

Fixtures are encoded by Google's protobuf runtime from descriptors declared in
tests/npds_pb.py; the product decodes them with its own wire-format reader.
The JSON path is the reference point: the same policy delivered either way
must compile to the same tables (stats equal) and NACK with the same error."""
import json

import pytest

import cilium_amd
import npds_pb
from cilium_amd import PolicyError, api, gen
from cilium_amd._lib import PROTO_HTTP, PROTO_KAFKA, PROTO_MEMCACHE

import nfa_cases


def npds_kafka_policy():
    rules = [{"api_key": 0, "api_version": 0, "topic": "orders"}, {"api_key": 3, "api_version": -1},
             {"api_key": -1, "api_version": -1, "client_id": "svc-a"}, {"topic": "t-0001", "api_key": 1}]
    return api.policy_set(api.network_policy("k", 7, ingress=[(9092, [api.port_rule(remote_policies=[5, 1], kafka=rules)])]))


def cases(kats):
    w2 = gen.http_workload(2, 200)
    return [
        ("http_kats", kats["http"]["policy"], [
            {"policy": 0, "port": c["conn"]["port"], "ingress": int(c["conn"]["ingress"]), "proto": PROTO_HTTP,
             "src_id": c["conn"]["src_id"], "dst_id": c["conn"]["dst_id"]} for c in kats["http"]["cases"]]),
        ("cfg2", w2.policy, w2.conns),
        ("memcache", gen.mc_policy(), gen.make_conns(8, 0, gen.MC_PORT, True, PROTO_MEMCACHE, 3000 + __import__("numpy").arange(8))),
        ("nfa", nfa_cases.policy(), nfa_cases.conns()),
        ("kafka_npds", npds_kafka_policy(), gen.make_conns(4, 0, 9092, True, PROTO_KAFKA, [1, 5, 6, 7])),
    ]


def compiled(load, policy_arg, conns):
    e = cilium_amd.Engine(-1)
    load(e, policy_arg)
    e.set_connections(conns)
    return e.stats(), e.nrules


@pytest.mark.parametrize("idx", range(5))
def test_proto_and_json_compile_identically(kats, idx):
    name, pol, conns = cases(kats)[idx]
    a = compiled(lambda e, p: e.update_policy(p), pol, conns)
    b = compiled(lambda e, p: e.update_policy_proto(p), npds_pb.discovery_response(pol), conns)
    assert a == b, name
    assert a[1] > 0


def test_policy_names_and_ids(kats):
    e = cilium_amd.Engine(-1)
    e.update_policy_proto(npds_pb.discovery_response(kats["http"]["policy"]))
    for i, p in enumerate(kats["http"]["policy"]["policies"]):
        assert e.policy_index(p["name"]) == i


def test_nack_keeps_previous_version_and_same_error(kats):
    d = kats["http"]["duplicate_port"]["policy"]
    with pytest.raises(PolicyError) as ej:
        cilium_amd.Engine(-1).update_policy(d)
    e = cilium_amd.Engine(-1)
    e.update_policy_proto(npds_pb.discovery_response(kats["http"]["policy"]))
    n0 = e.nrules
    with pytest.raises(PolicyError) as ep:
        e.update_policy_proto(npds_pb.discovery_response(d))
    assert str(ep.value) == str(ej.value)
    assert e.nrules == n0  # previous version in force


def bad_regex_policy():
    return api.policy_set(api.network_policy("b", 1, ingress=[(80, [api.port_rule(http=[{"headers": [
        {"name": ":path", "regex_match": "a**"}]}])])]))


def test_regex_error_text_matches_json():
    with pytest.raises(PolicyError) as ej:
        cilium_amd.Engine(-1).update_policy(bad_regex_policy())
    with pytest.raises(PolicyError) as ep:
        cilium_amd.Engine(-1).update_policy_proto(npds_pb.discovery_response(bad_regex_policy()))
    assert str(ep.value) == str(ej.value)


def test_malformed_wire_is_nacked(kats):
    good = npds_pb.discovery_response(kats["http"]["policy"])
    e = cilium_amd.Engine(-1)
    for bad in (good[:-3], good[:17], b"\x12\xff\xff\xff\xff\x0f", b"\x0b", b"\x12\x02\x0a"):
        with pytest.raises(PolicyError, match="NPDS"):
            e.update_policy_proto(bad)


def test_foreign_resource_type_is_nacked():
    R = npds_pb.cls("DiscoveryResponse")
    r = R(version_info="1")
    a = r.resources.add()
    a.type_url = "type.googleapis.com/envoy.api.v2.Listener"
    a.value = b""
    with pytest.raises(PolicyError, match="unexpected resource type"):
        cilium_amd.Engine(-1).update_policy_proto(r.SerializeToString())


def test_proto3_details():
    """Unknown fields skipped, unpacked repeated remotes accepted, the last
    oneof member wins, absent Kafka api_key reads as 0 (produce)."""
    NP = npds_pb.cls("NetworkPolicy")
    p = NP(name="x", policy=3)
    port = p.ingress_per_port_policies.add(port=80)
    r = port.rules.add()
    r.remote_policies.extend([9, 4])
    r.kafka_rules.kafka_rules.add(topic="t")
    r.http_rules.http_rules.add().headers.add(name=":path", regex_match="/a")  # oneof: replaces kafka_rules
    raw = p.SerializeToString()
    # unpacked remote_policies (field 1, varint) + an unknown field 77 (varint)
    raw += b"\x1a" + bytes([len(b"\x08\x07\x98\x04\x05")]) + b"\x08\x07\x98\x04\x05"  # port entry {port: 7, 77: 5}
    R = npds_pb.cls("DiscoveryResponse")
    resp = R(version_info="2")
    a = resp.resources.add()
    a.type_url = "type.googleapis.com/cilium.NetworkPolicy"
    a.value = raw
    e = cilium_amd.Engine(-1)
    e.update_policy_proto(resp.SerializeToString())
    js = {"policies": [{"name": "x", "policy": 3, "ingress_per_port_policies": [
        {"port": 80, "rules": [{"remote_policies": [4, 9], "http_rules": {"http_rules": [
            {"headers": [{"name": ":path", "regex_match": "/a"}]}]}}]}, {"port": 7, "rules": []}]}]}
    conns = [{"policy": 0, "port": 80, "ingress": 1, "proto": PROTO_HTTP, "src_id": 4, "dst_id": 1}]
    e.set_connections(conns)
    f = cilium_amd.Engine(-1)
    f.update_policy(js)
    f.set_connections(conns)
    assert e.stats() == f.stats() and e.nrules == f.nrules == 1
