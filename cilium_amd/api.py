"""Rule-model mirror of the reference (host side, no compute).

- PortRule / PortProtocol / L7Rules + sanitize(): the rule container and its
  validation, pkg/policy/api/rule_validation.go:232-357 (R0, K1, H1)

- PortRuleHTTP / PortRuleKafka: pkg/policy/api/http.go:28-60, kafka.go:26-107
- get_http_rule: pkg/envoy/server.go:336-399 (getHTTPRule) -> Envoy HeaderMatchers
- sort helpers:  pkg/envoy/sort.go:199-319 (SortHeaderMatchers,
                 SortHTTPNetworkPolicyRules)
- network_policy(): assembles the cilium.NetworkPolicy JSON the engine ingests
  (envoy/cilium/npds.proto:31-182).
"""
from dataclasses import dataclass, field
from functools import cmp_to_key
from typing import List, Optional


@dataclass
class PortRuleHTTP:
    path: str = ""
    method: str = ""
    host: str = ""
    headers: List[str] = field(default_factory=list)


@dataclass
class PortRuleKafka:
    role: str = ""
    api_key: str = ""
    api_version: str = ""
    client_id: str = ""
    topic: str = ""

    def to_json(self):
        d = {}
        if self.role:
            d["role"] = self.role
        if self.api_key:
            d["apiKey"] = self.api_key
        if self.api_version:
            d["apiVersion"] = self.api_version
        if self.client_id:
            d["clientID"] = self.client_id
        if self.topic:
            d["topic"] = self.topic
        return d


def get_http_rule(h: PortRuleHTTP):
    """getHTTPRule (pkg/envoy/server.go:336-399): list of HeaderMatcher dicts, or None."""
    headers = []
    if h.path:
        headers.append({"name": ":path", "regex_match": h.path})
    if h.method:
        headers.append({"name": ":method", "regex_match": h.method})
    if h.host:
        headers.append({"name": ":authority", "regex_match": h.host})
    for hdr in h.headers:
        strs = hdr.split(" ", 1)  # strings.SplitN(hdr, " ", 2)
        if len(strs) == 2:
            key = strs[0].rstrip(":")  # strings.TrimRight(strs[0], ":")
            headers.append({"name": key, "exact_match": strs[1]})
        else:
            headers.append({"name": strs[0], "present_match": True})
    if not headers:
        return None
    return sort_header_matchers(headers)


def _cmp(a, b):
    return (a > b) - (a < b)


def header_matcher_cmp(m1, m2):
    """HeaderMatcherLess (pkg/envoy/sort.go:224-313) as a 3-way compare."""
    for key in ("name", "exact_match", "regex_match"):
        c = _cmp(m1.get(key, "").encode(), m2.get(key, "").encode())
        if c:
            return c
    r1, r2 = m1.get("range_match"), m2.get("range_match")
    if (r1 is None) != (r2 is None):
        return -1 if r1 is None else 1
    if r1 is not None:
        c = _cmp(r1.get("start", 0), r2.get("start", 0)) or _cmp(r1.get("end", 0), r2.get("end", 0))
        if c:
            return c
    c = _cmp(bool(m1.get("present_match")), bool(m2.get("present_match")))
    if c:
        return c
    for key in ("prefix_match", "suffix_match"):
        c = _cmp(m1.get(key, "").encode(), m2.get(key, "").encode())
        if c:
            return c
    return _cmp(bool(m1.get("invert_match")), bool(m2.get("invert_match")))


def sort_header_matchers(headers):
    return sorted(headers, key=cmp_to_key(header_matcher_cmp))


def http_rule_cmp(r1, r2):
    """HTTPNetworkPolicyRuleLess (pkg/envoy/sort.go:199-219)."""
    h1, h2 = r1.get("headers") or [], r2.get("headers") or []
    c = _cmp(len(h1), len(h2))
    if c:
        return c
    for a, b in zip(h1, h2):
        c = header_matcher_cmp(a, b)
        if c:
            return c
    return 0


def sort_http_rules(rules):
    return sorted(rules, key=cmp_to_key(http_rule_cmp))


def http_rules_from_api(rules: List[PortRuleHTTP], sort: bool = True):
    """getPortNetworkPolicyRule's HTTP branch (pkg/envoy/server.go:505-515)."""
    out = []
    for r in rules:
        hs = get_http_rule(r)
        out.append({"headers": hs} if hs else {})
    return sort_http_rules(out) if sort else out


def port_rule(remote_policies: Optional[List[int]] = None, http=None, kafka=None, l7proto=None, l7=None):
    r = {}
    if remote_policies:
        r["remote_policies"] = sorted(remote_policies)
    if http is not None:
        r["http_rules"] = {"http_rules": http}
    if kafka is not None:
        r["kafka_rules"] = {"kafka_rules": [k.to_json() if isinstance(k, PortRuleKafka) else k for k in kafka]}
    if l7proto:
        r["l7_proto"] = l7proto
    if l7 is not None:
        r["l7_rules"] = {"l7_rules": [{"rule": x} for x in l7]}
    return r


def network_policy(name, policy_id=0, ingress=None, egress=None):
    """ingress/egress: list of (port, [port_rule...]) or dicts."""
    def ports(lst):
        out = []
        for p in lst or []:
            if isinstance(p, dict):
                out.append(p)
            else:
                port, rules = p
                out.append({"port": port, "protocol": "TCP", "rules": rules})
        return out
    return {"name": name, "policy": policy_id,
            "ingress_per_port_policies": ports(ingress),
            "egress_per_port_policies": ports(egress)}


def policy_set(*policies):
    return {"policies": list(policies)}


# ------------------------------------------------------------ rule container (R0)
# pkg/policy/api/kafka.go:153-197 (KafkaAPIKeyMap), :274-293 (roles)
KAFKA_API_KEYS = {
    "produce": 0, "fetch": 1, "offsets": 2, "metadata": 3, "leaderandisr": 4, "stopreplica": 5,
    "updatemetadata": 6, "controlledshutdown": 7, "offsetcommit": 8, "offsetfetch": 9, "findcoordinator": 10,
    "joingroup": 11, "heartbeat": 12, "leavegroup": 13, "syncgroup": 14, "describegroups": 15, "listgroups": 16,
    "saslhandshake": 17, "apiversions": 18, "createtopics": 19, "deletetopics": 20, "deleterecords": 21,
    "initproducerid": 22, "offsetforleaderepoch": 23, "addpartitionstotxn": 24, "addoffsetstotxn": 25,
    "endtxn": 26, "writetxnmarkers": 27, "txnoffsetcommit": 28, "describeacls": 29, "createacls": 30,
    "deleteacls": 31, "describeconfigs": 32, "alterconfigs": 33,
}
KAFKA_ROLES = {"produce": [0, 3, 18], "consume": [1, 2, 3, 8, 9, 10, 11, 12, 13, 14, 18]}
KAFKA_MAX_TOPIC_LEN = 255
MAX_PORTS = 40  # rule_validation.go:27


class SanitizeError(ValueError):
    pass


def _go_parse_int(s, base, bits, unsigned, fn):
    """strconv.ParseInt / ParseUint (Go 1.10: base 0 takes 0x / 0 prefixes, no underscores)."""
    def err(what):
        return SanitizeError(f'strconv.{fn}: parsing "{s}": {what}')
    t = s
    neg = False
    if not unsigned and t[:1] in ("+", "-"):
        neg, t = t[0] == "-", t[1:]
    if not t:
        raise err("invalid syntax")
    b = base
    if b == 0:
        if t[:2].lower() == "0x":
            b, t = 16, t[2:]
            if not t:
                raise err("invalid syntax")
        elif t[0] == "0" and len(t) > 1:
            b, t = 8, t[1:]
        else:
            b = 10
    digits = "0123456789abcdefghijklmnopqrstuvwxyz"[:b]
    v = 0
    for ch in t.lower():
        if ch not in digits:
            raise err("invalid syntax")
        v = v * b + digits.index(ch)
    limit = (1 << bits) - 1 if unsigned else (1 << (bits - 1)) - (0 if neg else 1)
    if v > limit:
        raise err("value out of range")
    return -v if neg else v


def sanitize_kafka(k: PortRuleKafka):
    """PortRuleKafka.Sanitize (rule_validation.go:232-275)."""
    if k.api_key and k.role:
        raise SanitizeError(f'Cannot set both Role:"{k.role}" and APIKey :"{k.api_key}" together')
    if k.api_key and k.api_key.lower() not in KAFKA_API_KEYS:
        raise SanitizeError(f'invalid Kafka APIKey :"{k.api_key}"')
    if k.role and k.role.lower() not in KAFKA_ROLES:
        raise SanitizeError(f'invalid Kafka APIRole :"{k.role}"')
    if k.api_version:
        try:
            _go_parse_int(k.api_version, 10, 16, False, "ParseInt")
        except SanitizeError:
            raise SanitizeError(f'invalid Kafka APIVersion :"{k.api_version}"') from None
    if k.topic:
        if len(k.topic) > KAFKA_MAX_TOPIC_LEN:
            raise SanitizeError(f"kafka topic exceeds maximum len of {KAFKA_MAX_TOPIC_LEN}")
        # KafkaTopicValidChar = ^[a-zA-Z0-9\\._\\-]+$ (the doubled escape admits a backslash)
        if not all(c.isascii() and (c.isalnum() or c in "\\._-") for c in k.topic):
            raise SanitizeError(f'invalid Kafka Topic name "{k.topic}"')


def sanitize_http(h: PortRuleHTTP):
    """PortRuleHTTP.Sanitize (http.go:66-84): Path and Method must compile as
    Go regexps (checked with the product's Go-syntax parser); Host and
    headers are not checked there."""
    from . import _lib
    for pat in (h.path, h.method):
        if pat:
            _lib.debug_regex(pat, b"")  # raises ValueError with Go's error text


@dataclass
class PortProtocol:
    port: str = ""
    protocol: str = ""

    def sanitize(self):
        """PortProtocol.sanitize (rule_validation.go:338-357); normalises protocol."""
        if self.port == "":
            raise SanitizeError("Port must be specified")
        try:
            p = _go_parse_int(self.port, 0, 16, True, "ParseUint")
        except SanitizeError as e:
            raise SanitizeError(f"Unable to parse port: {e}") from None
        if p == 0:
            raise SanitizeError("Port cannot be 0")
        proto = (self.protocol or "ANY").upper()
        if proto not in ("TCP", "UDP", "ANY"):
            raise SanitizeError(f'invalid protocol "{proto}", must be {{ tcp | udp | any }}')
        self.protocol = proto


@dataclass
class L7Rules:
    http: Optional[List[PortRuleHTTP]] = None
    kafka: Optional[List[PortRuleKafka]] = None
    l7proto: str = ""
    l7: Optional[List[dict]] = None

    def is_empty(self):
        return self.http is None and self.kafka is None and self.l7 is None

    def sanitize(self):
        """L7Rules.sanitize (rule_validation.go:277-314)."""
        ntypes = 0
        if self.http is not None:
            ntypes += 1
            for h in self.http:
                sanitize_http(h)
        if self.kafka is not None:
            ntypes += 1
            for k in self.kafka:
                sanitize_kafka(k)
        if self.l7 is not None and not self.l7proto:
            raise SanitizeError("'l7' may only be specified when a 'l7proto' is also specified")
        if self.l7proto:
            ntypes += 1
            for r in self.l7 or []:
                if "" in r:  # PortRuleL7.Sanitize (l7.go:27-34)
                    raise SanitizeError("Empty key not allowed")
        if ntypes > 1:
            raise SanitizeError("multiple L7 protocol rule types specified in single rule")


@dataclass
class PortRule:
    ports: List[PortProtocol] = field(default_factory=list)
    rules: Optional[L7Rules] = None

    def sanitize(self):
        """PortRule.sanitize (rule_validation.go:316-336)."""
        if len(self.ports) > MAX_PORTS:
            raise SanitizeError(f"too many ports, the max is {MAX_PORTS}")
        has_l7 = self.rules is not None and not self.rules.is_empty()
        for p in self.ports:
            p.sanitize()
            if has_l7 and p.protocol != "TCP":
                raise SanitizeError(f"L7 rules can only apply exclusively to TCP, not {p.protocol}")
        if has_l7:
            self.rules.sanitize()

    def npds(self, remote_policies=None):
        """The NPDS per-port entries this (sanitized) rule contributes:
        [(port, protocol, [PortNetworkPolicyRule dict])] (pkg/envoy/server.go:
        getPortNetworkPolicyRule, :496-530)."""
        self.sanitize()
        out = []
        for p in self.ports:
            r = self.rules
            if r is None or r.is_empty():
                pr = port_rule(remote_policies)
            elif r.http is not None:
                pr = port_rule(remote_policies, http=http_rules_from_api(r.http))
            elif r.kafka is not None:
                pr = port_rule(remote_policies, kafka=r.kafka)
            else:
                pr = port_rule(remote_policies, l7proto=r.l7proto, l7=r.l7 or [])
            out.append((int(_go_parse_int(p.port, 0, 16, True, "ParseUint")), p.protocol, [pr]))
        return out
