"""Small synchronous calls on a multi-protocol engine (l7g_classify_host).

A call of at most kHostScanMax requests whose connections are all one
parser's (one Allowed(), one OnData) launches only that parser's kernel,
unpartitioned, behind a one-kernel copy of its inputs into HBM
(capi.cc:Classify, HostRun).  Every subset below -- one protocol, one
protocol plus unknown and parserless connections, every protocol at once,
a single request, zero-length requests -- must answer exactly as the oracle
does, and a call must not see a previous call's answers."""
import numpy as np
import pytest

from cilium_amd import gen

from test_gpu_http import assert_same

pytestmark = pytest.mark.gpu


def _subset(w, idx, extra_conns=()):
    idx = np.asarray(idx, np.int64)
    offs = np.concatenate([w.offsets[idx], w.offsets[idx[:len(extra_conns)]]])
    lens = np.concatenate([w.lengths[idx], w.lengths[idx[:len(extra_conns)]]])
    cids = np.concatenate([w.conn_ids[idx], np.asarray(extra_conns, np.uint32)])
    return gen.Workload(w.name + "-sub", w.arena, offs, lens, cids, w.conns, w.policy)


def test_small_calls_on_a_mixed_engine(engine, oracle):
    w = gen.mixed_workload(1200)
    conns = w.conns.copy()
    parserless = len(conns) - 1
    conns["proto"][parserless] = 0
    w = gen.Workload(w.name, w.arena, w.offsets, w.lengths, w.conn_ids, conns, w.policy)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    proto = conns["proto"][w.conn_ids]
    rng = np.random.default_rng(5)
    nc = len(conns)
    by = {p: np.nonzero(proto == p)[0] for p in np.unique(proto) if p != 0}
    assert len(by) >= 3, by.keys()
    cases = []
    for p, ix in by.items():
        for k in (1, 3, 17, 200):
            cases.append((f"p{p}x{k}", _subset(w, rng.choice(ix, min(k, len(ix)), replace=False))))
        cases.append((f"p{p}+unowned", _subset(w, rng.choice(ix, 20, replace=False), [nc + 7, 0xFFFFFFFF,
                                                                                      parserless])))
    allx = np.concatenate([v[:10] for v in by.values()])
    cases.append(("all", _subset(w, rng.permutation(allx))))
    cases.append(("unowned-only", _subset(w, [0, 1], [nc + 1, parserless])))
    for name, s in cases:
        got = engine.classify(s.arena, s.offsets, s.lengths, s.conn_ids)
        ref = oracle.classify_workload(s, 4)
        try:
            assert_same(got, ref, s)
        except AssertionError as e:
            raise AssertionError(f"{name}: {e}") from None


def test_single_request_calls_repeat(engine, oracle):
    """The latency path's shape: one request per call, many calls in a row,
    alternating protocols (the staging and device scratch are reused)."""
    w = gen.mixed_workload(400)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    ref = oracle.classify_workload(w, 4)
    for i in range(0, w.n, 3):
        v, r, c = engine.classify(w.arena, w.offsets[i:i + 1], w.lengths[i:i + 1], w.conn_ids[i:i + 1])
        assert (v[0], r[0], c[0]) == (ref[0][i], ref[1][i], ref[2][i]), (i, (v, r, c), (ref[0][i], ref[1][i], ref[2][i]))
