"""The HTTP latency kernel (one request per wave, its header lines framed
side by side; http_classify.hip:lat_request) against the oracle.

Calls of at most 64 requests take it (capi.cc kLatencyMax): every workload
below is cut into calls of 1..64 requests and each answer must equal the
oracle's -- the cfg1 / cfg2 streams, adversarial and chunked requests,
many rule sets (hot and general instantiations), and header blocks around the
kernel's line limit (63 lines side by side; more run sequentially)."""
import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import PROTO_HTTP

from test_gpu_http import assert_same, wl_from_reqs

pytestmark = pytest.mark.gpu


def _small_calls(engine, oracle, w, seed=3, nmax=64):
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    ref = oracle.classify_workload(w, 8)
    rng = np.random.default_rng(seed)
    got = [np.zeros(w.n, np.uint8), np.zeros(w.n, np.int32), np.zeros(w.n, np.uint32)]
    i = 0
    while i < w.n:
        k = int(rng.integers(1, nmax + 1))
        v, r, c = engine.classify(w.arena, w.offsets[i:i + k], w.lengths[i:i + k], w.conn_ids[i:i + k])
        got[0][i:i + k], got[1][i:i + k], got[2][i:i + k] = v, r, c
        i += k
    assert_same(tuple(got), ref, w)


@pytest.mark.parametrize("cfg", [1, 2])
def test_latency_cfg_streams(engine, oracle, cfg):
    _small_calls(engine, oracle, gen.http_workload(cfg, 3000))


def test_latency_adversarial(engine, oracle):
    reqs = gen.http_adversarial(3000, 99)
    base = gen.http_workload(2, 1)
    rng = np.random.default_rng(5)
    w = wl_from_reqs(reqs, base.policy, base.conns, rng.integers(0, len(base.conns), len(reqs)))
    _small_calls(engine, oracle, w)


def test_latency_chunked(engine, oracle):
    reqs = gen.http_chunked(2000, 77)
    base = gen.http_workload(2, 1)
    rng = np.random.default_rng(6)
    w = wl_from_reqs(reqs, base.policy, base.conns, rng.integers(0, len(base.conns), len(reqs)))
    _small_calls(engine, oracle, w)


def test_latency_many_rulesets(engine, oracle):
    _small_calls(engine, oracle, gen.cfg4_workload(3000, nids=64, rules_total=64 * 20))


def test_latency_line_limit(engine, oracle):
    """Header blocks of 1..70 lines (the kernel frames up to 63 side by side),
    with the constrained headers first, last and repeated, complete and cut."""
    pol = gen.cfg2_policy()
    reqs = []
    for nh in list(range(0, 8)) + [30, 61, 62, 63, 64, 65, 70]:
        for variant in range(4):
            hdr = [b"X-F%d: v%d" % (j, j) for j in range(nh)]
            if variant == 1:
                hdr = [b"Host: svc-7.a", b"X-Token: 12"] + hdr
            elif variant == 2:
                hdr = hdr + [b"Host: svc-7.a", b"Host: svc-9.b", b"X-Token: 12"]
            elif variant == 3:
                hdr = hdr[: nh // 2] + [b"Content-Length: 3"] + hdr[nh // 2:] + [b"Host: svc-12.c"]
            head = b"GET /api/v1/svc7/x HTTP/1.1\r\n" + b"".join(h + b"\r\n" for h in hdr) + b"\r\n"
            body = b"abc" if variant == 3 else b""
            r = head + body
            reqs += [r, r[:-1], r[: len(r) // 2], r.replace(b"\r\n", b"\r\x01", 1) if nh else r + b"x"]
    # CR runs and bare CRs where lines end (each line ends at its first CR)
    reqs += [b"GET / HTTP/1.1\r\nHost: a\r\r", b"GET / HTTP/1.1\r\r", b"GET / HTTP/1.1\r\nA: b\r\n\r\r",
             b"GET / HTTP/1.1\r\nA: b\r\r\n\r\n", b"GET / HTTP/1.1\r\n\r\r\n", b"\r\n\r\n", b"\r",
             b"GET / HTTP/1.1\r\nHost: svc-7.a\r\nX-Token: 1\r\n\r", b"GET /a\rb HTTP/1.1\r\n\r\n"]
    conns = gen.make_conns(1, 0, 80, True, PROTO_HTTP, [7])
    w = wl_from_reqs(reqs, pol, conns)
    _small_calls(engine, oracle, w, nmax=8)
