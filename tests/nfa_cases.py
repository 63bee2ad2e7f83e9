"""Shared NFA-fallback workload: HTTP rules whose regexes blow up as DFAs
(each over the 4096-state budget on its own), and requests that hit and miss
them.  Used by the CPU compile test and the GPU parity test."""
import random

from cilium_amd import api, gen

PATH_RE = "/api/(a|b)*a(a|b){14}"
HOST_RE = "(x|y)*x(x|y){13}\\.example"
TOKEN_RE = "(?s).*z[^q]{12}"
INV_RE = "/inv/(a|b)*a(a|b){14}"
BIG_RE = "/big/(.*/)?(a|b)*a.{40}"  # many positions: . spans every rune


def policy():
    rules = [
        {"headers": [{"name": ":method", "regex_match": "GET"}, {"name": ":path", "regex_match": PATH_RE}]},
        {"headers": [{"name": ":authority", "regex_match": HOST_RE}]},
        {"headers": [{"name": "x-token", "regex_match": TOKEN_RE}, {"name": ":method", "regex_match": "PUT"}]},
        {"headers": [{"name": ":method", "regex_match": "POST"},
                     {"name": ":path", "regex_match": INV_RE, "invert_match": True}]},
        {"headers": [{"name": ":path", "regex_match": BIG_RE}]},
        {"headers": [{"name": ":path", "regex_match": "/static/.*"}]},
    ]
    return api.policy_set(api.network_policy("nfa", 1, ingress=[(80, [api.port_rule(http=rules)])]))


def _ab(rng, n, hit, a="a", b="b"):
    s = [rng.choice(a + b) for _ in range(n)]
    if len(s) >= 15:
        s[-15] = a if hit else b
    return "".join(s)


def requests(n, seed=7):
    rng = random.Random(seed)
    out = []
    for i in range(n):
        kind = rng.randrange(7)
        method = rng.choice(["GET", "PUT", "POST", "DELETE"])
        host = "svc.local"
        path = "/other"
        hdrs = []
        if kind == 0:
            path = "/api/" + _ab(rng, rng.randint(10, 40), rng.random() < 0.5)
        elif kind == 1:
            host = _ab(rng, rng.randint(12, 30), rng.random() < 0.5, "x", "y")
            host = host[:-1] + ".example" if rng.random() < 0.8 else host + ".exampl"
        elif kind == 2:
            tail = "".join(rng.choice("abzqé") for _ in range(rng.randint(8, 20)))
            hdrs.append(("X-Token" if rng.random() < 0.5 else "x-token", tail + rng.choice(["", " ", "\t "])))
            if rng.random() < 0.3:
                hdrs.append(("x-token", "z" + "a" * 12))  # second occurrence: never looked at
        elif kind == 3:
            path = "/inv/" + _ab(rng, rng.randint(10, 30), rng.random() < 0.5)
        elif kind == 4:
            path = "/big/" + rng.choice(["", "x/y/"]) + _ab(rng, rng.randint(1, 6), True) + \
                "".join(rng.choice("ab/é") for _ in range(rng.randint(35, 45)))
        elif kind == 5:
            path = "/static/" + "x" * rng.randint(0, 20)
        else:
            path = "/api/" + "é" * rng.randint(0, 20)
        lines = [f"{method} {path} HTTP/1.1", f"Host: {host}"] + [f"{k}: {v}" for k, v in hdrs]
        out.append(("\r\n".join(lines) + "\r\n\r\n").encode())
    return out


def conns():
    return [{"policy": 0, "port": 80, "ingress": 1, "proto": gen.PROTO_HTTP if hasattr(gen, "PROTO_HTTP") else 1,
             "src_id": 5, "dst_id": 1}]
