"""Pin the oracle (and the host-side rule translation) to the reference's own
known-answer tests (tests/golden/reference_kats.json, see make_golden.py)."""
import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, INCOMPLETE, PARSE_ERROR, PROTO_HTTP, PROTO_KAFKA, PROTO_MEMCACHE

VERDICT = {"ALLOW": ALLOW, "DENY": DENY}
VERDICT_ALL = {"ALLOW": ALLOW, "DENY": DENY, "INCOMPLETE": INCOMPLETE, "PARSE_ERROR": PARSE_ERROR}


def test_regex_kats(oracle, kats):
    for k in kats["regex"]:
        if "compile_error" in k:
            if k["compile_error"]:
                with pytest.raises(ValueError, match="missing argument to repetition operator"):
                    oracle.Regex(k["pattern"])
            else:
                oracle.Regex(k["pattern"])
            continue
        assert oracle.Regex(k["pattern"]).match(k["input"], k["anchored"]) == k["match"], k


def _http_one(oracle, policy, req, conn):
    pol = oracle.Policy(policy)
    c = {"policy": pol.names.get(conn["policy_name"], -1), "port": conn["port"], "ingress": int(conn["ingress"]),
         "proto": PROTO_HTTP, "src_id": conn["src_id"], "dst_id": conn["dst_id"]}
    b = req.encode()
    v, r, cons = pol.classify([c], np.frombuffer(b, np.uint8), [0], [len(b)], [0])
    return int(v[0]), int(r[0]), int(cons[0])


def test_http_kats(oracle, kats):
    h = kats["http"]
    assert len(h["cases"]) == 19
    for case in h["cases"]:
        v, r, cons = _http_one(oracle, h["policy"], case["request"], case["conn"])
        assert v == VERDICT[case["expect"]], case["name"]
        assert cons == (len(case["request"]) if v in (ALLOW, DENY) else 0)


def test_http_duplicate_port_rejected(oracle, kats):
    d = kats["http"]["duplicate_port"]
    with pytest.raises(ValueError, match="Duplicate port"):
        oracle.Policy(d["policy"])


def test_http_translation_kats(kats):
    for case in kats["http_translation"]["cases"]:
        r = case["rule"]
        got = api.get_http_rule(api.PortRuleHTTP(path=r.get("path", ""), method=r.get("method", ""),
                                                 host=r.get("host", ""), headers=r.get("headers", [])))
        assert got == case["expected"]


def kafka_policy(rules, src=None):
    return api.policy_set(api.network_policy("ep", 1, ingress=[(9092, [api.port_rule(kafka=rules)])]))


def test_kafka_kats(oracle, kats):
    K = kats["kafka"]
    for case in K["cases"]:
        req = bytes.fromhex(K["requests"][case["request"]])
        pol = oracle.Policy(kafka_policy(case["rules"]))
        c = {"policy": 0, "port": 9092, "ingress": 1, "proto": PROTO_KAFKA, "src_id": case.get("src_id", 7), "dst_id": 9}
        v, r, cons = pol.classify([c], np.frombuffer(req, np.uint8), [0], [len(req)], [0])
        assert int(v[0]) == VERDICT[case["expect"]], case
        assert int(cons[0]) == len(req)


def test_kafka_empty_rule_list_is_wildcard_free(oracle):
    # rules.Kafka == nil (no group admits the identity) => deny (pkg/proxy/kafka.go:139-142)
    pol = oracle.Policy(api.policy_set(api.network_policy(
        "ep", 1, ingress=[(9092, [api.port_rule(remote_policies=[5], kafka=[{}])])])))
    req = gen.k_request(18, 0, 1, "c", b"")
    c = {"policy": 0, "port": 9092, "ingress": 1, "proto": PROTO_KAFKA, "src_id": 6, "dst_id": 9}
    v, _, _ = pol.classify([c], np.frombuffer(req, np.uint8), [0], [len(req)], [0])
    assert v[0] == DENY
    c["src_id"] = 5
    v, r, _ = pol.classify([c], np.frombuffer(req, np.uint8), [0], [len(req)], [0])
    assert v[0] == ALLOW and r[0] == 0


def memcache_policy(M, l7_rules):
    t = M["policy_template"]
    return api.policy_set(api.network_policy(t["name"], t["policy"], ingress=[
        (t["port"], [api.port_rule(remote_policies=t["remote_policies"], l7proto=t["l7_proto"], l7=l7_rules)])]))


def _mc_conn(pol, M):
    c = M["conn"]
    return {"policy": pol.names[c["policy_name"]], "port": c["port"], "ingress": int(c["ingress"]),
            "proto": PROTO_MEMCACHE, "src_id": c["src_id"], "dst_id": c["dst_id"]}


def test_memcache_kats(oracle, kats):
    M = kats["memcache"]
    assert len(M["cases"]) == 31
    for case in M["cases"]:
        pol = oracle.Policy(memcache_policy(M, case["l7_rules"]))
        for chk in case["checks"]:
            b = bytes.fromhex(M["requests"][chk["request"]])
            v, r, cons = pol.classify([_mc_conn(pol, M)], np.frombuffer(b, np.uint8), [0], [len(b)], [0])
            assert VERDICT_ALL[chk["expect"]] == int(v[0]), (case["name"], chk)
            assert int(cons[0]) == chk["consumed"], (case["name"], chk)


def test_memcache_wrong_remote_denied(oracle, kats):
    M = kats["memcache"]
    pol = oracle.Policy(memcache_policy(M, [{"command": "set"}]))
    b = bytes.fromhex(M["requests"]["setHelloText"])
    c = _mc_conn(pol, M)
    c["src_id"] = 2  # not in remote_policies 1/3/4
    v, _, _ = pol.classify([c], np.frombuffer(b, np.uint8), [0], [len(b)], [0])
    assert v[0] == DENY


@pytest.mark.parametrize("rule,msg", [
    ({"command": "set", "bogus": "x"}, "Unsupported key: bogus"),
    ({"keyExact": "k"}, "command not specified but key was provided"),
    ({"command": "nosuch", "keyPrefix": "k"}, "command not specified but key was provided"),
    ({"command": "get", "keyRegex": "a**"}, "invalid nested repetition operator"),
])
def test_memcache_rule_parse_errors(oracle, kats, rule, msg):
    # memcache.L7RuleParser (proxylib/memcached/parser.go:114-148): ParseError => policy NACK
    with pytest.raises(ValueError, match=msg):
        oracle.Policy(memcache_policy(kats["memcache"], [rule]))
