"""The NFA fallback on the GPU: rule sets with regexes over the DFA state
budget (each compiled to a bit-parallel rune NFA, evaluated by the pre-pass
kernel), bit-exact against the oracle's Pike VM.  Mixed with DFA-evaluated
matchers, inverted matchers, absent / repeated / OWS-padded headers, hot
(LDS) and cold (HBM) rule-set images."""
import numpy as np
import pytest

import nfa_cases
from cilium_amd import gen
from cilium_amd._lib import ALLOW, DENY
from test_gpu_http import assert_same, wl_from_reqs

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("n", [64, 5000])
def test_nfa_rules_parity(engine, oracle, n):
    pol = nfa_cases.policy()
    reqs = nfa_cases.requests(n, seed=n)
    w = wl_from_reqs(reqs, pol, nfa_cases.conns())
    engine.update_policy(pol)
    engine.set_connections(w.conns)
    assert engine.stats()["http_nfas"] == 5
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    ref = oracle.classify_workload(w, 8)
    assert_same(got, ref, w)
    v, r = got[0], got[1]
    assert (v == ALLOW).sum() > n // 10 and (v == DENY).sum() > n // 10
    if n >= 5000:  # every NFA rule allows something
        assert len(set(r[v == ALLOW].tolist())) == 6


def test_nfa_rules_cold_image(engine, oracle):
    """Two rule sets (two ports): the less used one runs from HBM."""
    pol = nfa_cases.policy()
    pol["policies"][0]["ingress_per_port_policies"].append(
        dict(pol["policies"][0]["ingress_per_port_policies"][0], port=8080))
    reqs = nfa_cases.requests(3000, seed=3)
    conns = nfa_cases.conns() + [dict(nfa_cases.conns()[0], port=8080, src_id=6)]
    ids = np.array([0 if i % 5 else 1 for i in range(len(reqs))], np.uint32)
    w = wl_from_reqs(reqs, pol, conns, ids)
    engine.update_policy(pol)
    engine.set_connections(w.conns)
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 8), w)


THOUSAND_RE = "(a|b)*a.{1000}"  # every repeat count Go accepts (<= 1000): 1003 NFA positions, no DFA


def _thousand_value(rng, hit):
    # 'a' exactly 1001 runes before the end <=> match (unanchored: some suffix)
    head = "".join(rng.choice("ab") for _ in range(rng.randint(0, 20)))
    tail = "".join(rng.choice("abé/") for _ in range(1000))
    return head + ("a" if hit else "b") + tail if rng.random() < 0.8 else head + tail[:rng.randint(900, 999)]


def test_thousand_repeat_regexes(engine, oracle):
    """Go accepts `(a|b)*a.{1000}` (repeat counts <= 1000, pkg/policy/api/http.go:66-84
    compiles it): as an HTTP :path regex and a memcached keyRegex it is
    enforced on the device (bit-parallel NFA), bit-exact against the oracle."""
    import random
    from cilium_amd import api
    from cilium_amd._lib import PROTO_MEMCACHE
    rng = random.Random(11)
    http_rules = [{"headers": [{"name": ":path", "regex_match": "/k/" + THOUSAND_RE}]}]
    mc = [{"command": "get", "keyRegex": "^k" + THOUSAND_RE}]
    pol = api.policy_set(
        api.network_policy("t", 1, ingress=[(80, [api.port_rule(http=http_rules)])]),
        api.network_policy("m", 2, ingress=[(11211, [api.port_rule(l7proto="memcache", l7=mc)])]))
    reqs, ids = [], []
    for i in range(600):
        v = _thousand_value(rng, rng.random() < 0.5)
        if i % 2:
            reqs.append(f"GET /k/{v} HTTP/1.1\r\nHost: h\r\n\r\n".encode())
            ids.append(0)
        else:
            reqs.append(b"get k" + v.replace("/", "c").encode() + b"\r\n")
            ids.append(1)
    conns = [{"policy": 0, "port": 80, "ingress": 1, "proto": 1, "src_id": 5, "dst_id": 1},
             {"policy": 1, "port": 11211, "ingress": 1, "proto": PROTO_MEMCACHE, "src_id": 5, "dst_id": 1}]
    w = wl_from_reqs(reqs, pol, conns, np.array(ids, np.uint32))
    engine.update_policy(pol)
    engine.set_connections(w.conns)
    st = engine.stats()
    assert st["http_nfas"] == 1 and st["mc_nfas"] == 1
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 8), w)
    assert (got[0] == ALLOW).sum() > 100 and (got[0] == DENY).sum() > 100
