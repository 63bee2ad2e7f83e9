"""Concurrent submission (SURVEY.md §8(b) threading row): host-buffer calls
from several threads (each thread its own stream and staging) and device
calls on several torch streams (each stream its own partition scratch) on one
engine give the oracle's verdicts, bit-exact; calls on different streams that
share one counters array lose no hit (the reduce adds atomically)."""
import threading

import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW

from test_gpu_http import assert_same

pytestmark = pytest.mark.gpu


def slices(w, k):
    cut = np.linspace(0, w.n, k + 1).astype(int)
    return [np.arange(cut[i], cut[i + 1]) for i in range(k)]


def test_host_calls_from_threads(engine, oracle):
    w = gen.mixed_workload(40000)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    ref = oracle.classify_workload(w, 8)
    parts = slices(w, 6)
    errors, done = [], []

    def worker(idx):
        try:
            for rep in range(4):
                got = engine.classify(w.arena, w.offsets[idx], w.lengths[idx], w.conn_ids[idx])
                assert_same(got, tuple(r[idx] for r in ref))
            done.append(len(idx))
        except Exception as e:  # surfaced below
            errors.append(e)

    ts = [threading.Thread(target=worker, args=(p,)) for p in parts]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=120)
    assert not errors, errors[0]
    assert sum(done) == w.n


def test_device_calls_on_streams(engine, oracle):
    import torch
    w = gen.mixed_workload(30000, seed=77)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    ref = oracle.classify_workload(w, 8)
    dev = torch.device("cuda", 0)
    arena = torch.from_numpy(w.arena).to(dev)
    parts = slices(w, 3)
    streams = [torch.cuda.Stream() for _ in parts]
    nrules = engine.nrules
    counters = torch.zeros(nrules + 8, dtype=torch.int64, device=dev)  # shared by every stream
    outs = []
    for p, s in zip(parts, streams):
        d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
             (w.offsets[p].view(np.int64), w.lengths[p].view(np.int32), w.conn_ids[p].view(np.int32))]
        o = [torch.empty(len(p), dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
        outs.append((d, o))
    torch.cuda.synchronize()
    for rep in range(3):
        for (d, o), p, s in zip(outs, parts, streams):
            engine.classify_device(arena.data_ptr(), arena.numel(), d[0].data_ptr(), d[1].data_ptr(), d[2].data_ptr(),
                                   len(p), o[0].data_ptr(), o[1].data_ptr(), o[2].data_ptr(),
                                   counters_ptr=counters.data_ptr(), stream=s.cuda_stream)
    torch.cuda.synchronize()
    v, r = ref[0], ref[1]
    cnt = counters.cpu().numpy()
    hits = np.bincount(r[(v == ALLOW) & (r >= 0)], minlength=nrules)[:nrules]
    np.testing.assert_array_equal(cnt[:nrules], 3 * hits)
    np.testing.assert_array_equal(cnt[nrules:nrules + 5], 3 * np.bincount(v, minlength=5)[:5])
    for (d, o), p in zip(outs, parts):
        got = (o[0].cpu().numpy(), o[1].cpu().numpy(), o[2].cpu().numpy().view(np.uint32))
        assert_same(got, tuple(r[p] for r in ref))
