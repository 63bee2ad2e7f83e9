"""Regexes past the register NFA (> 1,024 positions) on the GPU: Go 1.10 accepts
every repeat count <= 1000 (pkg/policy/api/http.go:66-84 compiles the HTTP
header regexes with it; proxylib/memcached/parser.go:89-95 the keyRegex;
proxylib/cassandra/cassandraparser.go:89,113 the query_table regex;
proxylib/r2d2/r2d2parser.go the file regex), so `.{1000}x.{1000}` and
`(a|b)*a.{1000}b.{1000}` must be enforced, not refused.  Their DFAs exceed any
budget and their NFAs have ~2,000 positions: they run as large NFAs (sparse
follow rows, state sets in per-lane scratch, regex/nfa_walk.h nfa_run_big),
bit-exact against the oracle's Pike VM, on HTTP :path, memcached keyRegex,
cassandra query_table and r2d2 file."""
import random

import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, PROTO_CASSANDRA, PROTO_HTTP, PROTO_MEMCACHE, PROTO_R2D2
from test_gpu_http import assert_same, wl_from_reqs

pytestmark = pytest.mark.gpu

PATS = [".{1000}x.{1000}", "(a|b)*a.{1000}b.{1000}"]


def _value(rng, which):
    """About half match: a planted a..x / a..b pair exactly 1001 runes apart
    with at least 1000 runes after it."""
    n = rng.choice([1500, 2001, 2002, 2003, 2100, 2600])
    v = [rng.choice("abcyé") for _ in range(n)]
    if rng.random() < 0.5:
        k = rng.randrange(0, max(1, n - 2001))
        v[k] = "a"
        if k + 1001 < n:
            v[k + 1001] = "x" if which == 0 else "b"
    return "".join(v)


def _policy(pat):
    http = [{"headers": [{"name": ":path", "regex_match": "/k/" + pat}]}]
    mc = [{"command": "get", "keyRegex": "^k" + pat}]
    cs = [{"query_action": "select", "query_table": pat}]
    r2 = [{"cmd": "READ", "file": pat}]
    return api.policy_set(
        api.network_policy("h", 1, ingress=[(80, [api.port_rule(http=http)])]),
        api.network_policy("m", 2, ingress=[(11211, [api.port_rule(l7proto="memcache", l7=mc)])]),
        api.network_policy("c", 3, ingress=[(gen.CASS_PORT, [api.port_rule(l7proto="cassandra", l7=cs)])]),
        api.network_policy("r", 4, ingress=[(gen.R2D2_PORT, [api.port_rule(l7proto="r2d2", l7=r2)])]))


CONNS = [{"policy": 0, "port": 80, "ingress": 1, "proto": PROTO_HTTP, "src_id": 5, "dst_id": 1},
         {"policy": 1, "port": 11211, "ingress": 1, "proto": PROTO_MEMCACHE, "src_id": 5, "dst_id": 1},
         {"policy": 2, "port": gen.CASS_PORT, "ingress": 1, "proto": PROTO_CASSANDRA, "src_id": 5, "dst_id": 1},
         {"policy": 3, "port": gen.R2D2_PORT, "ingress": 1, "proto": PROTO_R2D2, "src_id": 5, "dst_id": 1}]


def _path_value(rng, which):
    """Matched from the value's start (HTTP: the whole value): about half match."""
    hit = rng.random() < 0.5
    body = lambda k: "".join(rng.choice("abcyé") for _ in range(k))  # noqa: E731
    if which == 0:
        v = body(1000) + ("x" if hit else "c") + body(1000)
    else:
        v = "".join(rng.choice("ab") for _ in range(rng.randint(0, 8))) + "a" + body(1000) + ("b" if hit else "c") + body(1000)
    return v if rng.random() < 0.8 else v[:-1]


def _request(kind, v):
    if kind == 0:
        return f"GET /k/{v} HTTP/1.1\r\nHost: h\r\n\r\n".encode()
    if kind == 1:
        return b"get k" + v.replace(" ", "c").encode() + b"\r\n"
    if kind == 2:
        return gen.cass_query_frame("select * from " + v.replace(" ", "c"))
    return b"READ " + v.replace(" ", "c").encode() + b"\r\n"


@pytest.mark.parametrize("which", [0, 1])
def test_large_nfa_every_protocol(engine, oracle, which):
    pat = PATS[which]
    rng = random.Random(17 + which)
    reqs, ids = [], []
    for i in range(800):
        kind = i % 4
        # (the HTTP value and the memcached key, after "^k", are matched from their start)
        reqs.append(_request(kind, _path_value(rng, which) if kind < 2 else _value(rng, which)))
        ids.append(kind)
    pol = _policy(pat)
    w = wl_from_reqs(reqs, pol, CONNS, np.array(ids, np.uint32))
    engine.update_policy(pol)  # compiles: no refusal
    engine.set_connections(w.conns)
    st = engine.stats()
    assert st["http_nfas"] == 1 and st["mc_nfas"] == 1
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 8), w)
    for kind in range(4):  # every protocol both allows and denies
        v = got[0][np.array(ids) == kind]
        assert (v == ALLOW).sum() > 40 and (v == DENY).sum() > 40, (kind, np.bincount(v))
