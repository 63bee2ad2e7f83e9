"""Rule-model mirror of the reference (host side, no compute).

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
