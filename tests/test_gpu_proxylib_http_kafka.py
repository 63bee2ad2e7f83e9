"""The proxylib "http" and "kafka" parsers on the GPU, through the C-ABI
(OpenModule / OnNewConnection / OnData / Close).

Both are registered next to "memcache" (proxylib/proxylib/parserfactory.go:
68-71) with the rule parsers PortNetworkPolicyRule_HttpRules / _KafkaRules
(policymap.go:42-45); their connections use proxylib's policymap semantics
(policymap.go:150-236: installed entries only, no port entry => drop, SrcId as
the remote in both directions, connection.go:176-179).  The expected verdicts
are the oracle's under those semantics; where they coincide with the
reference's own known answers (the Envoy integration verdicts for ingress,
pkg/kafka/policy_test.go, pkg/proxy/kafka_test.go) the test checks those too.
"""
import struct

import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd import proxylib as P
from cilium_amd._lib import ALLOW, DENY, PROTO_HTTP, PROTO_KAFKA

pytestmark = pytest.mark.gpu

PROXYLIB = 4  # L7G_CONN_PROXYLIB
DENIED_403 = (b"HTTP/1.1 403 Forbidden\r\ncontent-length: 15\r\ncontent-type: text/plain\r\n\r\n"
              b"Access denied\r\n")


@pytest.fixture(scope="module")
def module():
    mid = P.open_module([("node-id", "host~127.0.0.1~proxylib-http-kafka~localdomain")])
    assert mid != 0
    yield mid
    P.close_module(mid)


def oracle_px(oracle, policy, proto, port, ingress, src, dst, reqs, pol_index=0):
    conns = gen.make_conns(1, pol_index, port, ingress, proto, [src], dst)
    conns["flags"] = PROXYLIB
    arena, offs, lens = gen.pack(reqs)
    return oracle.Policy(policy).classify(conns, arena, offs, lens, np.zeros(len(reqs), np.uint32))


def test_http_kats_through_proxylib(module, oracle, kats):
    h = kats["http"]
    P.policy_update(module, h["policy"])
    names = [p["name"] for p in h["policy"]["policies"]]
    for i, case in enumerate(h["cases"]):
        cc = case["conn"]
        req = case["request"].encode()
        c = P.Connection(module, "http", 100 + i, cc["ingress"], cc["src_id"], cc["dst_id"], "1.1.1.1:34567",
                         "10.1.1.1:%d" % cc["port"], cc["policy_name"], 1024)
        assert c.result == P.OK
        res, ops = c.on_data(False, [req], 4)
        assert res == P.OK
        pidx = names.index(cc["policy_name"]) if cc["policy_name"] in names else -1
        v, r, cons = oracle_px(oracle, h["policy"], PROTO_HTTP, cc["port"], cc["ingress"], cc["src_id"],
                               cc["dst_id"], [req], pidx)
        want = P.PASS if v[0] == ALLOW else P.DROP
        assert ops == [(want, len(req))], (case["name"], ops)
        if cc["ingress"]:  # SrcId is the remote on ingress in both filters: the Envoy verdicts hold
            assert v[0] == (ALLOW if case["expect"] == "ALLOW" else DENY), case["name"]
        inj = c.take_inject(True)
        assert inj == (DENIED_403 if want == P.DROP else b"")
        res, ops = c.on_data(True, [b"HTTP/1.1 200 OK\r\ncontent-length: 0\r\n\r\n"], 4)
        assert res == P.OK and ops == [(P.PASS, 38)]
        c.close()


def test_http_pipelined_one_launch_matches_oracle(module, oracle):
    """Many pipelined requests in one OnData call: one op per request, each the
    oracle's verdict and length (frames proposed by the host, decided on the
    device in one launch)."""
    w = gen.http_workload(2, 300)
    reqs = [bytes(w.arena[int(o):int(o) + int(n)]) for o, n in zip(w.offsets, w.lengths)]
    reqs[7] = reqs[7][:-2] + b"Content-Length: 3\r\n\r\nabc"  # a body
    P.policy_update(module, w.policy)
    c = P.Connection(module, "http", 501, True, 1000, 7, "1.1.1.1:2", "10.0.0.1:80", "10.0.0.1", 16384)
    assert c.result == P.OK
    res, ops = c.on_data(False, [b"".join(reqs)], len(reqs) + 2)
    assert res == P.OK
    v, r, cons = oracle_px(oracle, w.policy, PROTO_HTTP, 80, True, 1000, 7, reqs)
    want = [(P.PASS if x == ALLOW else P.DROP, len(q)) for x, q in zip(v, reqs)]
    assert ops == want
    assert (v == ALLOW).any() and (v == DENY).any()
    inj = c.take_inject(True)
    # Inject copies what fits (connection.go:190-203): the buffer fills up
    assert inj == (DENIED_403 * int((v == DENY).sum()))[:16384]
    c.close()


def kafka_policy(rules, port=9092):
    return api.policy_set(api.network_policy("ep", 1, ingress=[(port, [api.port_rule(kafka=rules)])]))


def decode_produce_resp_v0(b):
    size, corr, nt = struct.unpack(">iii", b[:12])
    assert size == len(b) - 4
    p, out = 12, []
    for _ in range(nt):
        n = struct.unpack(">h", b[p:p + 2])[0]
        name = b[p + 2:p + 2 + n].decode()
        p += 2 + n
        np_ = struct.unpack(">i", b[p:p + 4])[0]
        p += 4
        parts = []
        for _ in range(np_):
            pid, err, off = struct.unpack(">ihq", b[p:p + 14])
            p += 14
            parts.append((pid, err, off))
        out.append((name, parts))
    assert p == len(b)
    return corr, out


def test_kafka_kats_through_proxylib(module, oracle, kats):
    K = kats["kafka"]
    for i, case in enumerate(K["cases"]):
        req = bytes.fromhex(K["requests"][case["request"]])
        pol = kafka_policy(case["rules"])
        P.policy_update(module, pol)
        src = case.get("src_id", 7)
        c = P.Connection(module, "kafka", 200 + i, True, src, 9, "1.1.1.1:4000", "10.0.0.2:9092", "ep", 4096)
        assert c.result == P.OK
        res, ops = c.on_data(False, [req], 4)
        assert res == P.OK
        v, r, cons = oracle_px(oracle, pol, PROTO_KAFKA, 9092, True, src, 9, [req])
        want = P.PASS if v[0] == ALLOW else P.DROP
        assert ops == [(want, len(req))], (case, ops)
        if case["rules"]:  # a non-empty rule list: proxylib and the Go proxy agree (MatchesRule)
            assert v[0] == (ALLOW if case["expect"] == "ALLOW" else DENY), case
        inj = c.take_inject(True)
        if want == P.DROP and req[4:6] == b"\x00\x00":  # produce: the deny response names the partitions
            corr, topics = decode_produce_resp_v0(inj) if req[6:8] == b"\x00\x00" else (None, None)
            if corr is not None:
                assert corr == struct.unpack(">i", req[8:12])[0]
                assert topics and all(err == 29 for _, parts in topics for _, err, _ in parts)
        c.close()


def test_kafka_deny_response_disallowed_topic(module):
    """pkg/proxy/kafka_test.go:184-258: a produce to "disallowedTopic" under the
    rules {metadata v0} + {produce v0 allowedTopic} is answered with
    ErrTopicAuthorizationFailed (errno 29) for its partition."""
    rules = [api.PortRuleKafka(api_key="metadata", api_version="0"),
             api.PortRuleKafka(api_key="produce", api_version="0", topic="allowedTopic")]
    P.policy_update(module, kafka_policy(rules))
    c = P.Connection(module, "kafka", 300, True, 200, 9, "1.1.1.1:4000", "10.0.0.2:9092", "ep", 4096)
    msgs = [gen.k_message(b"first"), gen.k_message(b"second")]
    ok = gen.k_produce(0, 41, "tester", [("allowedTopic", [(0, msgs)])])
    bad = gen.k_produce(0, 42, "tester", [("disallowedTopic", [(0, msgs)])])
    res, ops = c.on_data(False, [ok + bad], 4)
    assert res == P.OK and ops == [(P.PASS, len(ok)), (P.DROP, len(bad))]
    corr, topics = decode_produce_resp_v0(c.take_inject(True))
    assert corr == 42 and topics == [("disallowedTopic", [(0, 29, 0)])]
    c.close()


def test_kafka_pipelined_one_launch_matches_oracle(module, oracle):
    w = gen.kafka_workload(400, seed=1234)
    reqs = [bytes(w.arena[int(o):int(o) + int(n)]) for o, n in zip(w.offsets, w.lengths)]
    P.policy_update(module, w.policy)
    c = P.Connection(module, "kafka", 401, True, 2000, 9, "1.1.1.1:4000", "10.0.0.1:9092", "10.0.0.1", 1 << 16)
    assert c.result == P.OK
    stream = b"".join(reqs)
    res, ops = c.on_data(False, [stream[:5000], stream[5000:]], len(reqs) + 2)
    assert res == P.OK
    v, r, cons = oracle_px(oracle, w.policy, PROTO_KAFKA, 9092, True, 2000, 9, reqs)
    want = [(P.PASS if x == ALLOW else P.DROP, len(q)) for x, q in zip(v, reqs)]
    assert ops == want
    assert (v == ALLOW).any() and (v == DENY).any()
    # partial frame: MORE with the missing byte count from the size prefix
    res, ops = c.on_data(False, [reqs[0][:7]], 4)
    assert res == P.OK and ops == [(P.MORE, len(reqs[0]) - 7)]
    c.close()


def test_unknown_parser_still_rejected(module):
    c = P.Connection(module, "cassandra-not-here", 601, True, 1, 2, "1.1.1.1:1", "2.2.2.2:80", "x", 64)
    assert c.result == P.UNKNOWN_PARSER
