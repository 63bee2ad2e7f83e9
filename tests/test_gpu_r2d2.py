"""r2d2 on the GPU: the r2d2 kernel bit-exact against the oracle (random
lines: every cmd, extra / leading spaces, stray CR, missing CRLF, an
NFA-fallback file regex, remote-restricted groups, the port-0 entry), alone
and mixed with HTTP; and the reference's proxylib op sequences
(proxylib/r2d2/r2d2parser_test.go:64-180) through OnData."""
import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd import proxylib as P
from test_gpu_http import assert_same, wl_from_reqs

pytestmark = pytest.mark.gpu


def test_r2d2_parity(engine, oracle):
    w = gen.r2d2_workload(40000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 8), w)
    assert len(set(got[1].tolist())) == 8  # every rule, incl. the NFA one and port 0, allows something


def test_r2d2_mixed_with_http(engine, oracle):
    r = gen.r2d2_workload(3000, nconns=16)
    h = gen.http_workload(2, 3000, nconns=16)
    pol = {"policies": r.policy["policies"] + [dict(h.policy["policies"][0], name="http")]}
    conns = np.concatenate([r.conns, h.conns])
    conns["policy"][16:] = 1
    reqs = [bytes(r.arena[int(o):int(o) + int(n)]) for o, n in zip(r.offsets, r.lengths)] + \
           [bytes(h.arena[int(o):int(o) + int(n)]) for o, n in zip(h.offsets, h.lengths)]
    ids = np.concatenate([r.conn_ids, h.conn_ids + 16])
    perm = np.random.default_rng(3).permutation(len(reqs))
    w = wl_from_reqs([reqs[i] for i in perm], pol, conns, ids[perm])
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 8), w)


def test_reference_op_sequences():
    mid = P.open_module([("node-id", "host~127.0.0.1~r2d2~localdomain")])
    try:
        def conn(cid, name):
            c = P.Connection(mid, "r2d2", cid, True, 1, 2, "1.1.1.1:34567", "2.2.2.2:80", name, 256)
            assert c.result == P.OK
            return c
        c = conn(1, "no-policy")  # TestR2d2OnDataIncomplete
        assert c.on_data(False, [b"READ xssss"], 4) == (P.OK, [(P.MORE, 1)])
        c.close()
        P.policy_update(mid, api.policy_set(api.network_policy("cp1", 2, ingress=[(80, [{"l7_proto": "r2d2"}])])))
        c = conn(2, "cp1")  # TestR2d2OnDataBasicPass
        msgs = [b"READ sssss\r\n", b"WRITE sssss\r\n", b"HALT\r\n", b"RESET\r\n"]
        assert c.on_data(False, [b"".join(msgs)], 8) == (P.OK, [(P.PASS, len(m)) for m in msgs] + [(P.MORE, 1)])
        c.close()
        c = conn(3, "cp1")  # TestR2d2OnDataMultipleReq
        assert c.on_data(False, [b"RE", b"SET\r\n"], 4) == (P.OK, [(P.PASS, 7), (P.MORE, 1)])
        c.close()
        for name, rule, msgs in (("cp2", {"cmd": "READ"}, [b"READ xssss\r\n", b"WRITE xssss\r\n"]),  # AllowDenyCmd
                                 ("cp3", {"file": "s.*"}, [b"READ ssss\r\n", b"WRITE yyyyy\r\n"])):  # AllowDenyRegex
            P.policy_update(mid, api.policy_set(api.network_policy(name, 2, ingress=[(80, [api.port_rule(
                l7proto="r2d2", l7=[rule])])])))
            c = conn(4, name)
            assert c.on_data(False, [b"".join(msgs)], 4) == (P.OK, [(P.PASS, len(msgs[0])), (P.DROP, len(msgs[1])),
                                                                     (P.MORE, 1)])
            assert c.take_inject(True) == b"ERROR\r\n"
            c.close()
    finally:
        P.close_module(mid)
