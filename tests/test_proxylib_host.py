"""proxylib C-ABI (include/proxylib_abi.h) without a GPU: module instances,
connection registration errors and the no-fallback rule
(proxylib/proxylib.go:57-155, connection.go:65-101, instance.go:85-143)."""
import os

import pytest

from cilium_amd import proxylib as P


@pytest.fixture()
def host_module(monkeypatch):
    monkeypatch.setenv("L7G_DEVICE", "-1")  # compile-only engine: no verdicts
    mid = P.open_module([("node-id", "host-test-%d" % os.getpid())])
    assert mid != 0
    yield mid
    P.close_module(mid)


def test_open_module_params():
    assert P.open_module([("bogus", "x")]) == 0


def test_open_module_refcount(monkeypatch):
    monkeypatch.setenv("L7G_DEVICE", "-1")
    a = P.open_module([("node-id", "n1"), ("access-log-path", "/tmp/l")])
    b = P.open_module([("node-id", "n1"), ("access-log-path", "/tmp/l")])
    c = P.open_module([("node-id", "n2"), ("access-log-path", "/tmp/l")])
    assert a == b != 0 and c not in (0, a)
    for m in (a, b, c):
        P.close_module(m)


def test_no_gpu_no_module(monkeypatch):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    monkeypatch.delenv("L7G_DEVICE", raising=False)
    assert P.open_module([("node-id", "needs-a-gpu")]) == 0  # fails loudly: no CPU verdict path


@pytest.mark.parametrize("proto,dst,exp", [
    ("memcache", "2.2.2.2:80", P.OK),
    ("memcache", "[::1]:11211", P.OK),
    ("http", "2.2.2.2:80", P.OK),
    ("kafka", "2.2.2.2:9092", P.OK),
    ("cassandra-not-here", "2.2.2.2:80", P.UNKNOWN_PARSER),
    ("memcache", "2.2.2.2", P.INVALID_ADDRESS),
    ("memcache", "2.2.2.2:0", P.INVALID_ADDRESS),
    ("memcache", "2.2.2.2:http", P.INVALID_ADDRESS),
    ("memcache", "::1:80", P.INVALID_ADDRESS),
    ("memcache", "2.2.2.2:4294967296", P.INVALID_ADDRESS),
])
def test_on_new_connection(host_module, proto, dst, exp):
    n0 = P.connections()
    c = P.Connection(host_module, proto, 77, True, 1, 2, "1.1.1.1:34567", dst, "bm1", 30)
    assert c.result == exp
    assert P.connections() == n0 + (1 if exp == P.OK else 0)
    if exp == P.OK:
        c.close()
        assert P.connections() == n0


def test_invalid_instance_and_unknown_connection():
    c = P.Connection(987654, "memcache", 78, True, 1, 2, "1.1.1.1:1", "2.2.2.2:80", "bm1")
    assert c.result == P.INVALID_INSTANCE
    assert P.on_data(424242, False, [b"get a\r\n"], 4)[0] == P.UNKNOWN_CONNECTION


def test_reply_without_request_is_parser_error(host_module):
    # text parser reply path indexes replyQueue[0] (text/parser.go:201): empty => panic => PARSER_ERROR
    c = P.Connection(host_module, "memcache", 79, True, 1, 2, "1.1.1.1:1", "2.2.2.2:80", "bm1", 30)
    res, ops = c.on_data(True, [b"STORED\r\n"], 4)
    assert res == P.PARSER_ERROR and ops == []
    c.close()


def test_request_needs_the_device(host_module):
    c = P.Connection(host_module, "memcache", 80, True, 1, 2, "1.1.1.1:1", "2.2.2.2:80", "bm1", 30)
    assert c.on_data(False, [b"get a\r\n"], 4)[0] == P.UNKNOWN_ERROR  # no CPU verdict fallback
    # NOP before the parser is chosen, MORE without a CRLF (no verdict needed)
    c2 = P.Connection(host_module, "memcache", 81, True, 1, 2, "1.1.1.1:1", "2.2.2.2:80", "bm1", 30)
    assert c2.on_data(False, [b""], 4) == (P.OK, [])
    assert c2.on_data(False, [b"get a\r"], 4) == (P.OK, [(P.MORE, 1)])
    c.close()
    c2.close()


def _mixed_port_policy(rules, protocol="TCP"):
    from cilium_amd import api
    return api.policy_set(api.network_policy("bm1", 3, ingress=[{"port": 80, "protocol": protocol, "rules": rules}]))


def _mc_rule(cmd="get"):
    from cilium_amd import api
    return api.port_rule(l7proto="memcache", l7=[{"command": cmd}])


def test_mismatched_l7_types_nack(host_module):
    """newPortNetworkPolicyRules panics with ParseError on a second, different
    registered parser on one port (proxylib/proxylib/policymap.go:135-143);
    Instance.PolicyUpdate recovers it as the update's error and keeps the old
    map (instance.go:168-219)."""
    from cilium_amd import api
    good = _mixed_port_policy([_mc_rule()])
    P.policy_update(host_module, good)
    r2 = api.port_rule(l7proto="r2d2", l7=[{"cmd": "READ"}])
    with pytest.raises(ValueError, match="Mismatching L7 types on the same port"):
        P.policy_update(host_module, _mixed_port_policy([_mc_rule(), r2]))
    http = api.port_rule(http=[{"headers": [{"name": ":path", "regex_match": "/a"}]}])
    with pytest.raises(ValueError, match="Mismatching L7 types"):
        P.policy_update(host_module, _mixed_port_policy([http, _mc_rule()]))


def test_unregistered_parser_before_mismatch_is_drop_all_not_nack(host_module):
    """An unregistered parser returns the port as drop-all before any later rule
    is looked at (policymap.go:128-134), so no mismatch is seen after it; a
    rule without L7 (type name "") never mismatches; UDP ports are never parsed
    by proxylib (:206-209)."""
    from cilium_amd import api
    unknown = api.port_rule(l7proto="no-such-parser", l7=[{"x": "y"}])
    r2 = api.port_rule(l7proto="r2d2", l7=[{"cmd": "READ"}])
    P.policy_update(host_module, _mixed_port_policy([_mc_rule(), unknown, r2]))
    P.policy_update(host_module, _mixed_port_policy([api.port_rule(remote_policies=[7]), _mc_rule()]))
    P.policy_update(host_module, _mixed_port_policy([_mc_rule(), r2], protocol="UDP"))


def test_envoy_view_accepts_mismatched_l7_types():
    """Envoy's NPDS has no such check (envoy/cilium_network_policy.h:150-165):
    the batch API installs the same version."""
    from cilium_amd import api
    from cilium_amd.engine import Engine
    r2 = api.port_rule(l7proto="r2d2", l7=[{"cmd": "READ"}])
    e = Engine(-1)  # L7G_HOST_ONLY: compile-only engine
    e.update_policy(_mixed_port_policy([_mc_rule(), r2]))
    e.close()
