"""memcached rule loading and rule-set compilation on the host (no GPU):
the product's policy loader accepts / rejects exactly what the oracle (and
memcache.L7RuleParser, proxylib/memcached/parser.go:114-148) does."""
import pytest

import cilium_amd
from cilium_amd import api, gen
from cilium_amd._lib import PROTO_MEMCACHE
from cilium_amd.engine import PolicyError

from test_oracle_kats import memcache_policy


@pytest.fixture(scope="module")
def host():
    return cilium_amd.Engine(-1)  # L7G_HOST_ONLY: compiler only


@pytest.mark.parametrize("rule,msg", [
    ({"command": "set", "bogus": "x"}, "Unsupported key: bogus"),
    ({"keyExact": "k"}, "command not specified but key was provided"),
    ({"command": "nosuch", "keyPrefix": "k"}, "command not specified but key was provided"),
    ({"command": "get", "keyRegex": "a**"}, "invalid nested repetition operator"),
])
def test_rule_errors_match_oracle(host, oracle, kats, rule, msg):
    pol = memcache_policy(kats["memcache"], [rule])
    with pytest.raises(ValueError, match=msg):
        oracle.Policy(pol)
    with pytest.raises(PolicyError, match=msg):
        host.update_policy(pol)


def test_rules_after_unknown_parser_are_not_parsed(host, oracle):
    pol = api.policy_set(api.network_policy("mc", 1, ingress=[(11211, [
        api.port_rule(l7proto="no.such.parser", l7=[{"file": "x"}]),
        api.port_rule(l7proto="memcache", l7=[{"keyExact": "k"}])])]))
    oracle.Policy(pol)
    host.update_policy(pol)


def test_kat_policies_compile(host, kats):
    M = kats["memcache"]
    for case in M["cases"]:
        host.update_policy(memcache_policy(M, case["l7_rules"]))
        host.set_connections(gen.make_conns(1, 0, 80, True, PROTO_MEMCACHE, [1]))
        st = host.stats()
        assert st["mc_rulesets"] == 1 and st["mc_rules"] == len(case["l7_rules"])


def test_cfg5_rule_sets(host):
    w = gen.memcache_workload(100)
    host.update_policy(w.policy)
    host.set_connections(w.conns)
    st = host.stats()
    # in-group remotes on 11211 (8 mc rules + version), out-of-group (version), port-0 fallback for
    # 11212 (in-group and out-of-group identities both reach the wildcard entry)
    assert st["mc_rulesets"] == 3
    assert st["mc_dfas"] == 1
