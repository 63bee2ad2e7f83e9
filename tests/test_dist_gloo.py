"""Multi-process path on CPU (gloo, world_size 2): policy broadcast, identical
compiled tables on every rank, connection sharding, counter all-reduce
(SURVEY.md §8(e)).  The GPU path uses the same functions over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    import torch
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    sys.path.insert(0, os.path.join(root, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cilium_amd
        import refpy
        from cilium_amd import dist as l7dist, gen
        # policy known only to rank 0 (the NPDS receiver)
        w = gen.memcache_workload(6000, nconns=64) if rank == 0 else None
        pol = l7dist.broadcast_policy(w.policy if rank == 0 else None, dist)
        w = gen.memcache_workload(6000, nconns=64)  # same synthetic stream on every rank
        host = cilium_amd.Engine(-1)
        host.update_policy(pol)
        host.set_connections(w.conns)
        st = host.stats()
        owner, idx = l7dist.shard_by_connection(w.conn_ids, w.lengths, len(w.conns), world)
        mine = w.subset(idx[rank])
        # per-rank counters from this rank's shard (the oracle stands in for the
        # device verdicts here: CPU test of the exchange, not of the kernel)
        v, r, _ = refpy.Policy(pol).classify(mine.conns, mine.arena, mine.offsets, mine.lengths, mine.conn_ids)
        nr = host.nrules
        c = torch.zeros(nr + 8, dtype=torch.int64)
        c[nr:nr + 5] = torch.from_numpy(np.bincount(v, minlength=5)[:5].astype(np.int64))
        hit = r[r >= 0]
        c[:nr] = torch.from_numpy(np.bincount(hit, minlength=nr)[:nr].astype(np.int64))
        l7dist.allreduce_counters(c, dist)
        q.put((rank, pol, (st["mc_rulesets"], st["mc_rules"], st["mc_dfa_states"]), owner.tolist(),
               [len(x) for x in idx], c.numpy().tolist(), int(mine.lengths.astype(np.int64).sum())))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_gloo_world2_policy_shard_counters():
    world, port = 2, _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=240) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    (r0, pol0, st0, own0, n0, c0, b0), (r1, pol1, st1, own1, n1, c1, b1) = res
    assert pol0 == pol1 and st0 == st1 and own0 == own1 and c0 == c1
    # every request on exactly one rank; contiguous connection ranges; bytes balanced
    assert n0[0] + n0[1] == 6000 and n0[0] > 0 and n0[1] > 0
    assert own0 == sorted(own0)
    assert abs(b0 - b1) / (b0 + b1) < 0.2
    # all-reduced counters equal the unsharded verdict histogram
    import sys
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import refpy
    from cilium_amd import gen
    w = gen.memcache_workload(6000, nconns=64)
    v, r, _ = refpy.classify_workload(w)
    nr = len(c0) - 8
    assert c0[nr:nr + 5] == np.bincount(v, minlength=5)[:5].tolist()
    assert sum(c0[:nr]) == int((r >= 0).sum())
