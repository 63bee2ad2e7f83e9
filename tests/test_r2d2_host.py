"""r2d2 (proxylib/r2d2/r2d2parser.go) on the host: the rule parser's NACKs in
the product loader, and the oracle against the reference's own test cases
(proxylib/r2d2/r2d2parser_test.go:64-180)."""
import numpy as np
import pytest

import cilium_amd
from cilium_amd import PolicyError, api, gen
from cilium_amd._lib import ALLOW, DENY, INCOMPLETE, PROTO_R2D2


def pol(l7=None, name="cp"):
    r = api.port_rule(l7proto="r2d2", l7=l7) if l7 is not None else {"l7_proto": "r2d2"}
    return api.policy_set(api.network_policy(name, 2, ingress=[(80, [r])]))


@pytest.mark.parametrize("rule,err", [
    ({"cmd": "JUMP"}, "NPDS: Unable to parse L7 r2d2 rule with invalid cmd: 'JUMP'"),
    ({"cmd": "HALT", "file": "x"}, "NPDS: Unable to parse L7 r2d2 rule, cmd 'HALT' is not compatible with 'file'"),
    ({"path": "/"}, "NPDS: Unsupported key: path"),
    ({"file": "a**"}, "regexp: Compile(`a**`): error parsing regexp: invalid nested repetition operator: `**`"),
])
def test_rule_parser_nacks(rule, err):
    with pytest.raises(PolicyError) as e:
        cilium_amd.Engine(-1).update_policy(pol([rule]))
    assert str(e.value) == err


def test_rule_parser_accepts():
    e = cilium_amd.Engine(-1)
    e.update_policy(pol([{"cmd": "READ", "file": "s.*"}, {"cmd": "WRITE"}, {"file": ""}, {}]))
    e.set_connections(gen.make_conns(1, 0, 80, True, PROTO_R2D2, [1]))
    assert e.stats()["r2d2_rules"] == 4


def run(oracle, policy, reqs, src=1):
    conns = gen.make_conns(1, 0, 80, True, PROTO_R2D2, [src])
    arena, offs, lens = gen.pack(reqs)
    return oracle.Policy(policy).classify(conns, arena, offs, lens, np.zeros(len(reqs), np.uint32))


def test_reference_cases(oracle):
    # TestR2d2OnDataIncomplete (:64-68): no policy for the connection, no CRLF -> MORE 1
    v, r, c = run(oracle, api.policy_set(), [b"READ xssss"])
    assert (v[0], c[0]) == (INCOMPLETE, 1)
    # TestR2d2OnDataBasicPass (:70-96): l7_proto r2d2 without rules passes everything
    msgs = [b"READ sssss\r\n", b"WRITE sssss\r\n", b"HALT\r\n", b"RESET\r\n"]
    v, r, c = run(oracle, pol(), msgs)
    assert list(v) == [ALLOW] * 4 and list(c) == [len(m) for m in msgs]
    # TestR2d2OnDataAllowDenyCmd (:117-146)
    v, r, c = run(oracle, pol([{"cmd": "READ"}]), [b"READ xssss\r\n", b"WRITE xssss\r\n"])
    assert list(v) == [ALLOW, DENY] and list(c) == [12, 13]
    # TestR2d2OnDataAllowDenyRegex (:148-180)
    v, r, c = run(oracle, pol([{"file": "s.*"}]), [b"READ ssss\r\n", b"WRITE yyyyy\r\n"])
    assert list(v) == [ALLOW, DENY] and list(c) == [11, 13]
