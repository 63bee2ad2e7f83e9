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
