"""cassandra (proxylib/cassandra/cassandraparser.go) on the host: the rule
parser's NACKs (CassandraRuleParser, :99-134) in the product loader against
the oracle loader, and the compiled rule-set shape."""
import pytest

import cilium_amd
from cilium_amd import PolicyError, api, gen
from cilium_amd._lib import PROTO_CASSANDRA


def pol(l7, name="cp"):
    return api.policy_set(api.network_policy(name, 2, ingress=[(80, [api.port_rule(l7proto="cassandra", l7=l7)])]))


@pytest.mark.parametrize("rule,err", [
    ({"query_action": "selectx"}, "NPDS: Unable to parse L7 cassandra rule with invalid query_action: 'selectx'"),
    ({"query_action": "create-role", "query_table": "x"},
     "NPDS: query_action 'create-role' is not compatible with a query_table match"),
    ({"table": "x"}, "NPDS: Unsupported key: table"),
    ({"query_table": "a**"}, "regexp: Compile(`a**`): error parsing regexp: invalid nested repetition operator: `**`"),
])
def test_rule_parser_nacks(oracle, rule, err):
    with pytest.raises(PolicyError) as e:
        cilium_amd.Engine(-1).update_policy(pol([rule]))
    assert str(e.value) == err
    with pytest.raises(ValueError):
        oracle.Policy(pol([rule]))


def test_rule_parser_accepts(oracle):
    rules = [{"query_action": "select", "query_table": "^ks\\."}, {"query_action": "grant-role"},
             {"query_table": ""}, {}, {"query_action": ""}]
    e = cilium_amd.Engine(-1)
    e.update_policy(pol(rules))
    e.set_connections(gen.make_conns(1, 0, 80, True, PROTO_CASSANDRA, [1]))
    oracle.Policy(pol(rules))


def test_workload_policy_compiles(oracle):
    w = gen.cassandra_workload(200)
    e = cilium_amd.Engine(-1)
    e.update_policy(w.policy)
    e.set_connections(w.conns)
    oracle.classify_workload(w)
