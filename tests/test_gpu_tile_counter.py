"""The HTTP kernels' tile counters across calls.

A batch of at least 2^18 HTTP requests on an HTTP-only engine takes its
tiles from a per-stream counter (capi.cc Classify).  Several such calls in a
row -- long requests (one tile per atomic), short ones (four per atomic),
and a small call in between (fixed stride) -- must each answer every request
exactly as the oracle does: a counter left non-zero would skip tiles."""
import numpy as np
import pytest

from cilium_amd import gen

from test_gpu_http import assert_same

pytestmark = pytest.mark.gpu


def _tiled(w, n):
    k = -(-n // w.n)
    idx = np.tile(np.arange(w.n), k)[:n]
    return gen.Workload(w.name + "-tiled", w.arena, w.offsets[idx], w.lengths[idx], w.conn_ids[idx], w.conns, w.policy)


@pytest.mark.timeout(600)
def test_counter_reset_between_calls(engine, oracle):
    big = gen.http_workload(2, 300000)  # 1.1 KB requests: one tile per atomic
    base = gen.select(big, np.arange(20000), "base")
    engine.update_policy(big.policy)
    engine.set_connections(big.conns)
    ref = oracle.classify_workload(big, 8)
    ref_small = tuple(x[:20000] for x in ref)
    short = [b"GET /a HTTP/1.1\r\nHost: svc-%d.x\r\n\r\n" % (i % 70) for i in range(4000)]
    arena, offs, lens = gen.pack(short)
    sw = gen.Workload("short", arena, offs, lens, big.conn_ids[:4000], big.conns, big.policy)
    ref_short_small = oracle.classify_workload(sw, 8)
    sbig = _tiled(sw, 280000)
    ref_sbig = tuple(np.concatenate([r] * 70)[:sbig.n] for r in ref_short_small)
    for _ in range(2):
        for w, r in ((big, ref), (sbig, ref_sbig), (big, ref)):
            got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
            assert_same(got, r, w)
        got = engine.classify(big.arena, big.offsets[:100], big.lengths[:100], big.conn_ids[:100])
        assert_same(got, tuple(x[:100] for x in ref_small))
