"""Rule-container validation (R0 / H1 / K1): api.PortRule.sanitize against
the reference's own test cases (pkg/policy/api/rule_validation_test.go), and
the Kafka Sanitize error cases on both the api mirror and the product's
policy loader (csrc/policy/policy.cc), which must NACK with the same text."""
import pytest

import cilium_amd
from cilium_amd import PolicyError, api
from cilium_amd.api import L7Rules, PortProtocol, PortRule, PortRuleHTTP, PortRuleKafka, SanitizeError

GET_ROOT = L7Rules(http=[PortRuleHTTP(method="GET", path="/")])


@pytest.mark.parametrize("ports,err", [
    ([("80", "TCP"), ("81", "TCP")], None),                                       # rule_validation_test.go:31-53
    ([("80", "UDP")], "L7 rules can only apply exclusively to TCP, not UDP"),       # :55-75
    ([("80", "ANY")], "L7 rules can only apply exclusively to TCP, not ANY"),       # :77-99
    ([("80", "TCP"), ("12345", "UDP")], "L7 rules can only apply exclusively to TCP, not UDP"),  # :101-123
    ([("80", "UDP"), ("12345", "TCP")], "L7 rules can only apply exclusively to TCP, not UDP"),  # :125-150
    ([("80", "")], "L7 rules can only apply exclusively to TCP, not ANY"),          # empty protocol parses as ANY
])
def test_l7_rules_with_non_tcp_protocols(ports, err):
    r = PortRule([PortProtocol(p, q) for p, q in ports], GET_ROOT)
    if err is None:
        r.sanitize()
    else:
        with pytest.raises(SanitizeError, match="^" + err + "$"):
            r.sanitize()


def test_l4_only_rules_take_any_protocol():
    PortRule([PortProtocol("53", "udp"), PortProtocol("80", "")]).sanitize()


@pytest.mark.parametrize("method,path", [("GET", "*"), ("*", "/")])  # TestHTTPRuleRegexes :155-203
def test_http_rule_regexes(method, path):
    r = PortRule([PortProtocol("80", "TCP"), PortProtocol("81", "TCP")],
                 L7Rules(http=[PortRuleHTTP(method=method, path=path)]))
    with pytest.raises(ValueError, match="missing argument to repetition operator"):
        r.sanitize()


def test_http_host_is_not_sanitized():
    PortRule([PortProtocol("80", "TCP")], L7Rules(http=[PortRuleHTTP(host="*")])).sanitize()


def test_l7_rules():  # TestL7Rules :278-352
    ports = [PortProtocol("80", "TCP"), PortProtocol("81", "TCP")]
    PortRule(ports, L7Rules(l7proto="test.lineparser", l7=[{"method": "PUT", "path": "/"},
                                                           {"method": "GET", "path": "/"}])).sanitize()
    PortRule(ports, L7Rules(l7proto="test.lineparser")).sanitize()
    with pytest.raises(SanitizeError, match="Empty key not allowed"):
        PortRule(ports, L7Rules(l7proto="test.lineparser", l7=[{"method": "PUT", "": "Foo"}])).sanitize()
    with pytest.raises(SanitizeError, match="'l7' may only be specified when a 'l7proto' is also specified"):
        PortRule(ports, L7Rules(l7=[{"a": "b"}])).sanitize()
    with pytest.raises(SanitizeError, match="multiple L7 protocol rule types specified in single rule"):
        PortRule(ports, L7Rules(http=[PortRuleHTTP(path="/")], kafka=[PortRuleKafka(topic="t")])).sanitize()
    with pytest.raises(SanitizeError, match="multiple L7 protocol rule types specified in single rule"):
        PortRule(ports, L7Rules(http=[], l7proto="memcache")).sanitize()


@pytest.mark.parametrize("port,err", [
    ("", "Port must be specified"), ("0", "Port cannot be 0"),
    ("65536", 'Unable to parse port: strconv.ParseUint: parsing "65536": value out of range'),
    ("http", 'Unable to parse port: strconv.ParseUint: parsing "http": invalid syntax'),
    ("0x50", None), ("010", None), ("-1", 'Unable to parse port: strconv.ParseUint: parsing "-1": invalid syntax'),
])
def test_port_protocol(port, err):
    p = PortProtocol(port, "TCP")
    if err is None:
        p.sanitize()
    else:
        with pytest.raises(SanitizeError, match="^" + err.replace("(", r"\(").replace(")", r"\)") + "$"):
            p.sanitize()


def test_port_protocol_values():
    with pytest.raises(SanitizeError, match='invalid protocol "SCTP", must be { tcp | udp | any }'):
        PortProtocol("80", "sctp").sanitize()
    assert PortRule([PortProtocol("0x50", "tcp")], GET_ROOT).npds()[0][:2] == (80, "TCP")
    with pytest.raises(SanitizeError, match="too many ports, the max is 40"):
        PortRule([PortProtocol(str(1000 + i), "TCP") for i in range(41)]).sanitize()


KAFKA_BAD = [
    (PortRuleKafka(role="produce", api_key="produce"), 'Cannot set both Role:"produce" and APIKey :"produce" together'),
    (PortRuleKafka(api_key="nosuchkey"), 'invalid Kafka APIKey :"nosuchkey"'),
    (PortRuleKafka(role="admin"), 'invalid Kafka APIRole :"admin"'),
    (PortRuleKafka(api_version="abc"), 'invalid Kafka APIVersion :"abc"'),
    (PortRuleKafka(api_version="40000"), 'invalid Kafka APIVersion :"40000"'),
    (PortRuleKafka(topic="t" * 256), "kafka topic exceeds maximum len of 255"),
    (PortRuleKafka(topic="bad topic"), 'invalid Kafka Topic name "bad topic"'),
    (PortRuleKafka(topic="bad/topic"), 'invalid Kafka Topic name "bad/topic"'),
]
KAFKA_GOOD = [PortRuleKafka(api_key="Produce", api_version="-1", topic="a.b_c-d\\e"), PortRuleKafka(role="CONSUME"),
              PortRuleKafka(topic="t" * 255), PortRuleKafka(api_version="+7")]


@pytest.mark.parametrize("rule,err", KAFKA_BAD)
def test_kafka_sanitize_errors_mirror_and_loader(rule, err):
    with pytest.raises(SanitizeError) as e:
        PortRule([PortProtocol("9092", "TCP")], L7Rules(kafka=[rule])).sanitize()
    assert str(e.value) == err
    pol = api.policy_set(api.network_policy("k", 1, ingress=[(9092, [api.port_rule(kafka=[rule])])]))
    with pytest.raises(PolicyError) as e2:
        cilium_amd.Engine(-1).update_policy(pol)
    assert str(e2.value) == err  # the product loader NACKs with Go's text


@pytest.mark.parametrize("rule", KAFKA_GOOD)
def test_kafka_sanitize_accepts(rule):
    PortRule([PortProtocol("9092", "TCP")], L7Rules(kafka=[rule])).sanitize()
    pol = api.policy_set(api.network_policy("k", 1, ingress=[(9092, [api.port_rule(kafka=[rule])])]))
    cilium_amd.Engine(-1).update_policy(pol)
