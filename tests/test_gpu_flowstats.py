"""Proxy statistics (l7g_flow_stats) on the GPU: per (policy, proto, port,
direction) received / forwarded / denied / error counts equal the aggregation
of the ORACLE's verdicts for the same stream (pkg/endpoint/endpoint.go:2207-2233
UpdateProxyStatistics), accumulate across calls and reset."""
import collections

import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, DENY, PARSE_ERROR

pytestmark = pytest.mark.gpu


def expected(w, v):
    out = collections.defaultdict(lambda: [0, 0, 0, 0])
    for cid, x in zip(w.conn_ids.tolist(), v.tolist()):
        if x > PARSE_ERROR or cid >= len(w.conns):
            continue
        c = w.conns[cid]
        if c["proto"] not in (1, 2, 3, 4, 5):
            continue
        k = (int(c["policy"]), int(c["proto"]), int(c["port"]), int(c["ingress"]))
        e = out[k]
        e[0] += 1
        e[1 if x == ALLOW else 2 if x == DENY else 3] += 1
    return {k: tuple(v) for k, v in out.items()}


def test_flow_stats_mixed(engine, oracle):
    w = gen.mixed_workload(60000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    engine.flow_stats_enable(True)
    try:
        engine.flow_stats(reset=True)
        engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
        want = expected(w, oracle.classify_workload(w, 8)[0])
        assert engine.flow_stats() == want
        assert len({k[1] for k in want}) == 3  # every protocol has flows
        engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
        twice = engine.flow_stats(reset=True)
        assert twice == {k: tuple(2 * x for x in t) for k, t in want.items()}
        assert engine.flow_stats() == {}
    finally:
        engine.flow_stats_enable(False)
