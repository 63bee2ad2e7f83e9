"""proxylib C-ABI on the GPU: the reference's memcached op sequences
(proxylib/proxylib_memcached_test.go:120-732) replayed through OpenModule /
OnNewConnection / OnData / Close, and pipelined streams checked against the
oracle frame by frame."""
import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd import proxylib as P
from cilium_amd._lib import PROTO_MEMCACHE, ALLOW, DENY

from test_oracle_kats import memcache_policy

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def module():
    mid = P.open_module([("access-log-path", "/tmp/l7g-access.sock")])
    assert mid != 0
    yield mid
    P.close_module(mid)


def test_memcache_op_sequences(module, kats):
    M, O = kats["memcache"], kats["memcache_ops"]
    cc = O["connection"]
    rules = {c["name"]: c["l7_rules"] for c in M["cases"]}
    assert len(O["calls"]) == 31
    for name, calls in O["calls"].items():
        P.policy_update(module, memcache_policy(M, rules[name]))
        n0 = P.connections()
        c = P.Connection(module, cc["proto"], cc["conn_id"], cc["ingress"], cc["src_id"], cc["dst_id"],
                         cc["src_addr"], cc["dst_addr"], cc["policy_name"], cc["inject_buf"])
        assert c.result == P.OK and P.connections() == n0 + 1
        for k in calls:
            exp_ops = [tuple(o) for o in k["ops"]]
            res, ops = c.on_data(k["reply"], [bytes.fromhex(b) for b in k["data"]], 1 + 2 * len(exp_ops))
            assert res == P.OK, (name, k)
            assert ops == exp_ops, (name, k, ops)
            buf, exp = c.take_inject(True), bytes.fromhex(k["inject"])
            assert buf == exp[:len(buf)], (name, buf, exp)
        c.close()
        assert P.connections() == n0


@pytest.mark.parametrize("binary", [False, True])
def test_pipelined_stream_matches_oracle(module, oracle, binary):
    """One OnData call carrying hundreds of pipelined requests: every PASS /
    DROP op and length equals the oracle's verdict for that frame."""
    reqs = [r for r in gen.memcache_requests(3000, 77) if (r[0] >= 0x80) == binary][:400]
    pol = gen.mc_policy()
    P.policy_update(module, pol)
    c = P.Connection(module, "memcache", 9, True, 3005, 7, "1.1.1.1:1", "2.2.2.2:%d" % gen.MC_PORT, "10.0.0.5", 1024)
    assert c.result == P.OK
    res, ops = c.on_data(False, [b"".join(reqs)], 2 * len(reqs) + 4)
    assert res == P.OK
    conns = gen.make_conns(1, 0, gen.MC_PORT, True, PROTO_MEMCACHE, [3005])
    conns["flags"] = 2 if binary else 1
    arena, offs, lens = gen.pack(reqs)
    v, r, cons = oracle.Policy(pol).classify(conns, arena, offs, lens, np.zeros(len(reqs), np.uint32))
    want = [(P.PASS if x == ALLOW else P.DROP, int(n)) for x, n in zip(v, cons)]
    assert set(v.tolist()) <= {ALLOW, DENY}
    assert ops[:len(reqs)] == want
    assert ops[len(reqs)] == (P.MORE, 24 if binary else 2)
    c.close()


def test_mismatched_l7_update_keeps_previous_policy(module):
    """A NACKed update (mismatching L7 types on one port, policymap.go:135-143)
    leaves the previous policy in force (instance.go:168-219): the connection
    still gets the old verdicts, where leaving the port out would drop."""
    from cilium_amd import api
    old = api.policy_set(api.network_policy("pm-nack", 3, ingress=[
        (11211, [api.port_rule(l7proto="memcache", l7=[{"command": "get"}])])]))
    P.policy_update(module, old)
    c = P.Connection(module, "memcache", 4242, True, 1, 2, "1.1.1.1:1", "2.2.2.2:11211", "pm-nack", 1024)
    assert c.result == P.OK
    req = b"get a\r\n"
    res, ops = c.on_data(False, [req], 4)
    assert res == P.OK and ops[0] == (P.PASS, len(req))
    bad = api.policy_set(api.network_policy("pm-nack", 3, ingress=[
        (11211, [api.port_rule(l7proto="memcache", l7=[{"command": "set"}]),
                 api.port_rule(l7proto="r2d2", l7=[{"cmd": "READ"}])])]))
    with pytest.raises(ValueError, match="Mismatching L7 types"):
        P.policy_update(module, bad)
    res, ops = c.on_data(False, [req], 4)
    assert res == P.OK and ops[0] == (P.PASS, len(req))  # still the old "get" rule
    c.close()
