"""The resident services (kernels/service.h, capi.cc Service): the
synchronous calls of l7g_classify_host whose requests are all HTTP (at most 8)
or all memcached (at most 64) are posted to a polling workgroup instead of
launched.  Their answers must be the launched path's and the oracle's, across
everything that stops or restarts a service: a policy update (new tables), a
connection update, a large batch that wants every CU, an idle exit, and calls
from several threads at once (one holds the service, the others launch)."""
import threading
import time

import numpy as np
import pytest

from cilium_amd import gen

pytestmark = pytest.mark.gpu


def _calls(w, proto, rng, count, maxn):
    """count calls of 1..maxn requests of one protocol (plus, in some, an
    unknown connection: still that protocol's call)."""
    p = w.conns["proto"][w.conn_ids]
    idx = np.nonzero(p == proto)[0]
    out = []
    for k in range(count):
        sel = rng.choice(idx, size=int(rng.integers(1, maxn + 1)), replace=False)
        cids = w.conn_ids[sel].copy()
        if k % 7 == 3:
            cids[-1] = len(w.conns) + 3  # unknown connection: answered UNSUPPORTED
        out.append((sel, cids))
    return out


def _check(engine, ref_pol, w, calls):
    """Each call as a drop-in makes it: its own requests packed into one small
    arena (the zero-copy / service size limits are on the call's bytes)."""
    for sel, cids in calls:
        arena, offs, lens = gen.pack([bytes(w.arena[int(o):int(o) + int(n)]) for o, n in
                                      zip(w.offsets[sel], w.lengths[sel])])
        got = engine.classify(arena, offs, lens, cids)
        want = ref_pol.classify(w.conns, arena, offs, lens, cids, 1)
        for g, r in zip(got, want):
            assert (g == r).all(), (sel, cids, got, want)


def test_service_calls_match_the_launched_path_and_the_oracle(engine, oracle):
    w = gen.mixed_workload(6000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    ref = oracle.Policy(w.policy)
    rng = np.random.default_rng(11)
    http = _calls(w, gen.PROTO_HTTP, rng, 120, 8)
    mc = _calls(w, gen.PROTO_MEMCACHE, rng, 120, 64)
    engine.service(True)
    _, s0 = engine.service()
    _check(engine, ref, w, http + mc)
    _, s1 = engine.service()
    # (a call whose one request is on an unknown connection uses no parser: launched)
    served = lambda calls: sum(1 for _, c in calls if (c < len(w.conns)).any())  # noqa: E731
    assert s1["http_calls"] - s0["http_calls"] == served(http)
    assert s1["mc_calls"] - s0["mc_calls"] == served(mc)
    assert s1["http_launches"] - s0["http_launches"] <= 2 and s1["mc_launches"] - s0["mc_launches"] <= 2
    # the launched path on the same calls
    engine.service(False)
    _check(engine, ref, w, http[:30] + mc[:30])
    _, s2 = engine.service(True)
    assert s2["http_calls"] == s1["http_calls"] and s2["mc_calls"] == s1["mc_calls"]


def test_service_restarts_after_updates_batches_and_idle(engine, oracle):
    w = gen.mixed_workload(6000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    engine.service(True)
    ref = oracle.Policy(w.policy)
    rng = np.random.default_rng(12)
    http = _calls(w, gen.PROTO_HTTP, rng, 20, 8)
    mc = _calls(w, gen.PROTO_MEMCACHE, rng, 20, 64)
    _check(engine, ref, w, http + mc)
    _, a = engine.service()
    # a policy update: new tables (cfg1's single rule for HTTP), the services restart on them
    pol2 = dict(w.policy)
    pol2["policies"] = [gen.http_workload(1, 10).policy["policies"][0]] + w.policy["policies"][1:]
    engine.update_policy(pol2)
    _check(engine, oracle.Policy(pol2), w, http + mc)
    _, b = engine.service()
    assert b["http_launches"] > a["http_launches"] and b["mc_launches"] > a["mc_launches"]
    engine.update_policy(w.policy)
    # a connection update (memcached connections switched to text-only framing)
    conns = w.conns.copy()
    conns["flags"][conns["proto"] == gen.PROTO_MEMCACHE] = 1
    engine.set_connections(conns)
    w2 = gen.Workload(w.name, w.arena, w.offsets, w.lengths, w.conn_ids, conns, w.policy)
    _check(engine, ref, w2, http + mc)
    engine.set_connections(w.conns)
    # a large batch between calls (the services leave so its persistent grids get every CU)
    big = gen.select(w, np.arange(w.n))
    v, r, c = engine.classify(big.arena, big.offsets, big.lengths, big.conn_ids)
    want = ref.classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids, 8)
    assert (v == want[0]).all() and (r == want[1]).all() and (c == want[2]).all()
    _check(engine, ref, w, http[:5] + mc[:5])
    # idle exit (~50 ms without a call), then a call starts it again
    _, c0 = engine.service()
    time.sleep(0.3)
    _check(engine, ref, w, http[:3] + mc[:3])
    _, c1 = engine.service()
    assert c1["http_launches"] > c0["http_launches"] and c1["mc_launches"] > c0["mc_launches"]


def test_service_calls_from_several_threads(engine, oracle):
    w = gen.mixed_workload(6000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    engine.service(True)
    ref = oracle.Policy(w.policy)
    errors = []

    def worker(seed):
        try:
            rng = np.random.default_rng(seed)
            calls = _calls(w, gen.PROTO_HTTP if seed % 2 else gen.PROTO_MEMCACHE, rng, 60, 8)
            _check(engine, ref, w, calls)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e)[:400])

    th = [threading.Thread(target=worker, args=(s,)) for s in range(6)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors
