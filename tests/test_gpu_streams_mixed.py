"""Large mixed batches (past 2^20 requests, every classifier, the partition
lists and work counters in use) on two caller streams, four calls in flight:
every verdict, rule id and consumed length, and the per-rule counters, equal
the oracle's -- calls in a row on one stream, and calls on two streams, do not
see each other's lists or counters.  At this size the memcached kernel runs on
the scratch set's side stream beside the Kafka kernel (capi.cc kBesideMin), so
the test also covers that fork / join with two caller streams in flight."""
import numpy as np
import pytest
import torch

from cilium_amd import gen

pytestmark = pytest.mark.gpu


def _tiled(w, n):
    k = -(-n // w.n)
    idx = np.tile(np.arange(w.n), k)[:n]
    return gen.Workload(w.name + "-tiled", w.arena, w.offsets[idx], w.lengths[idx], w.conn_ids[idx], w.conns, w.policy)


@pytest.mark.timeout(600)
def test_large_mixed_batches_on_two_streams(engine, oracle):
    u = gen.mixed_workload(200_000)
    ref_u = oracle.classify_workload(u, 8)
    w = _tiled(u, (1 << 20) + 4321)
    k = -(-w.n // u.n)
    ref = tuple(np.concatenate([r] * k)[:w.n] for r in ref_u)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(w.arena).to(dev)
    d_off = torch.from_numpy(w.offsets.view(np.int64)).to(dev)
    d_len = torch.from_numpy(w.lengths.view(np.int32)).to(dev)
    d_cid = torch.from_numpy(w.conn_ids.view(np.int32)).to(dev)
    nr = engine.nrules
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    outs = []
    torch.cuda.synchronize()  # the inputs are on the device before either stream reads them
    for call in range(4):
        s = streams[call % 2]
        with torch.cuda.stream(s):  # (the outputs' fills are ordered before the call on its stream)
            o = [torch.full((w.n,), 7, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
            cnt = torch.zeros(nr + 8, dtype=torch.int64, device=dev)
            engine.classify_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(),
                                   d_cid.data_ptr(), w.n, *[t.data_ptr() for t in o], counters_ptr=cnt.data_ptr(),
                                   stream=s.cuda_stream)
        outs.append((o, cnt))
    torch.cuda.synchronize()
    want_cnt = np.zeros(nr + 8, np.int64)
    allow = ref[0] == 1
    np.add.at(want_cnt, ref[1][allow], 1)
    for o, cnt in outs:
        v, r, c = o[0].cpu().numpy(), o[1].cpu().numpy(), o[2].cpu().numpy().view(np.uint32)
        bad = np.nonzero((v != ref[0]) | (r != ref[1]) | (c != ref[2]))[0]
        assert len(bad) == 0, (len(bad), bad[:8])
        got = cnt.cpu().numpy()
        assert (got[:nr] == want_cnt[:nr]).all()
