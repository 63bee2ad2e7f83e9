"""Requests no classifier owns still get a verdict, whatever kernels run.

An unknown connection index, a connection without a parser (proto 0, e.g.
after the proxylib shim's Close) and a request whose bytes leave the arena
are answered UNSUPPORTED, rule -1, consumed 0 -- in HTTP-only, Kafka-only,
memcached-only and mixed engines alike.  The host path reuses its device
scratch between calls, so a stale verdict from an earlier batch would show
here as a wrong answer (fail-open)."""
import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, UNSUPPORTED

from test_gpu_http import assert_same, both

pytestmark = pytest.mark.gpu


def _with_unowned(w, extra_conn_ids):
    """w plus requests (copies of w's first ones) on the given connection ids;
    connection 0 is turned into a parserless one."""
    k = len(extra_conn_ids)
    conns = w.conns.copy()
    conns["proto"][0] = 0
    return gen.Workload(w.name + "+unowned", w.arena, np.concatenate([w.offsets, w.offsets[:k]]),
                        np.concatenate([w.lengths, w.lengths[:k]]),
                        np.concatenate([w.conn_ids, np.asarray(extra_conn_ids, np.uint32)]), conns, w.policy)


@pytest.mark.parametrize("make", [
    lambda: gen.http_workload(2, 500),
    lambda: gen.kafka_workload(500),
    lambda: gen.memcache_workload(500),
    lambda: gen.mixed_workload(600),
], ids=["http", "kafka", "memcache", "mixed"])
def test_unowned_requests_answered(engine, oracle, make):
    w = make()
    # first a batch that allows a lot, so the host scratch holds ALLOW verdicts
    got0, _ = both(engine, oracle, w)
    assert (got0[0] == ALLOW).any()
    nc = len(w.conns)
    u = _with_unowned(w, [nc + 99, nc + 100, 0xFFFFFFFF, 0, 0])
    got, ref = both(engine, oracle, u)
    assert_same(got, ref, u)
    tail = got[0][-5:]
    assert (tail == UNSUPPORTED).all(), tail
    assert (got[1][-5:] == -1).all() and (got[2][-5:] == 0).all()


@pytest.mark.parametrize("make", [
    lambda: gen.http_workload(2, 64),
    lambda: gen.kafka_workload(64),
    lambda: gen.memcache_workload(64),
], ids=["http", "kafka", "memcache"])
def test_out_of_arena_requests(engine, make):
    """Offsets or lengths past the arena end are out of contract: UNSUPPORTED,
    and nothing beyond the arena is read (no fault)."""
    w = make()
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    n = w.n
    offs = w.offsets.copy()
    lens = w.lengths.copy()
    offs[0] = len(w.arena) + 4096          # starts past the end
    lens[1] = len(w.arena)                 # runs past the end
    offs[2] = np.uint64(1 << 62)           # far away
    v, r, c = engine.classify(w.arena, offs, lens, w.conn_ids)
    assert (v[:3] == UNSUPPORTED).all(), v[:3]
    assert (r[:3] == -1).all() and (c[:3] == 0).all()
    assert (v[3:n] != UNSUPPORTED).all()
