"""NPDS protobuf delivery on the GPU: verdicts, rule ids and consumed lengths
are bit-identical to the JSON delivery of the same policy (and so to the
oracle), for HTTP (cfg2 + the Envoy KATs), the NFA-fallback rules, memcached
through proxylib."""
import numpy as np
import pytest

import nfa_cases
import npds_pb
from cilium_amd import Engine, gen
from cilium_amd import proxylib as P
from test_gpu_http import assert_same, wl_from_reqs

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def engine_proto():
    return Engine(0)


@pytest.mark.parametrize("which", ["cfg2", "nfa"])
def test_proto_delivery_same_verdicts(engine, engine_proto, oracle, which):
    if which == "cfg2":
        w = gen.http_workload(2, 20000)
    else:
        w = wl_from_reqs(nfa_cases.requests(3000, seed=9), nfa_cases.policy(), nfa_cases.conns())
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    engine_proto.update_policy_proto(npds_pb.discovery_response(w.policy))
    engine_proto.set_connections(w.conns)
    a = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    b = engine_proto.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    for x, y in zip(a, b):
        assert np.array_equal(x, y)
    assert_same(b, oracle.classify_workload(w, 8), w)


def test_proxylib_memcache_proto_policy():
    mid = P.open_module([("node-id", "host~127.0.0.1~npds-proto~localdomain")])
    try:
        P.policy_update_proto(mid, npds_pb.discovery_response(gen.mc_policy()))
        c = P.Connection(mid, "memcache", 900, True, 3001, 5, "1.1.1.1:5000", "10.0.0.5:11211", "10.0.0.5", 512)
        assert c.result == P.OK
        res, ops = c.on_data(False, [b"get user:1\r\nget nope\r\n"], 4)
        assert res == P.OK and ops[:2] == [(P.PASS, 12), (P.DROP, 10)]
        c.close()
    finally:
        P.close_module(mid)
