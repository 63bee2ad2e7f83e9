"""Compiled tables broadcast from rank 0: rank 0
compiles the node's policy for every connection and broadcasts the compiled
image (cilium_amd/dist.py broadcast_tables over gloo here, RCCL on the box);
ranks > 0 install it without compiling a single rule set, and every rank's
device table blob is byte-identical to rank 0's and to a local compile."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _workload():
    from cilium_amd import gen
    return gen.mixed_workload(3000, seed=77)


def _worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cilium_amd
        from cilium_amd import dist as l7dist
        w = _workload()
        eng = cilium_amd.Engine(-1)
        image = l7dist.broadcast_tables(eng, dist, policy=w.policy if rank == 0 else None,
                                        conns=w.conns if rank == 0 else None)
        if rank != 0:
            eng.set_connections(w.conns)  # this rank's connection table: every rule set is in the image
        q.put((rank, len(image), eng.tables_digest, eng.tables_compiled, eng.nrules,
               {k: v for k, v in eng.stats().items() if k.endswith("rulesets")}))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3, 8])
def test_tables_broadcast(world):
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=500) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    import cilium_amd
    w = _workload()
    local = cilium_amd.Engine(-1)
    local.update_policy(w.policy)
    local.set_connections(w.conns)
    assert local.tables_compiled > 0
    r0 = res[0]
    assert r0[3] == local.tables_compiled  # rank 0 compiled what a lone engine compiles
    for rank, n, digest, compiled, nrules, st in res:
        assert digest == local.tables_digest, rank  # byte-identical installed tables
        assert nrules == local.nrules and st == r0[5]
        if rank:
            assert compiled == 0, (rank, compiled)  # installed, not compiled


def _nack_worker(rank, world, port, q):
    import sys
    import torch.distributed as dist
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import cilium_amd
        from cilium_amd import dist as l7dist
        w = _workload()
        eng = cilium_amd.Engine(-1)
        l7dist.broadcast_tables(eng, dist, policy=w.policy if rank == 0 else None,
                                conns=w.conns if rank == 0 else None)
        before = eng.tables_digest
        # rank 0 is handed a policy it must refuse (not even JSON): a NACK
        bad = "{not a policy"
        raised = None
        try:
            got = l7dist.broadcast_tables(eng, dist, policy=bad if rank == 0 else None)
        except cilium_amd.PolicyError as e:
            raised, got = type(e).__name__, None
        # the collective completed on every rank, and a later broadcast still works
        again = l7dist.broadcast_tables(eng, dist, policy=w.policy if rank == 0 else None,
                                        conns=w.conns if rank == 0 else None)
        q.put((rank, raised, got is None, before == eng.tables_digest, again is not None))
    finally:
        dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_tables_broadcast_nack_does_not_hang():
    """rank 0 refusing a policy must not leave the other ranks in
    the broadcast; every rank keeps its tables, rank 0 re-raises."""
    world = 3
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_nack_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted(q.get(timeout=250) for _ in range(world))
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, raised, got_none, kept, again in res:
        assert raised == ("PolicyError" if rank == 0 else None), (rank, raised)
        assert got_none and kept and again, (rank, got_none, kept, again)


def test_import_refuses_corrupt_image():
    import cilium_amd
    w = _workload()
    a = cilium_amd.Engine(-1)
    a.update_policy(w.policy)
    a.set_connections(w.conns)
    img = a.export_tables()
    b = cilium_amd.Engine(-1)
    for bad in (img[:len(img) // 2], b"x" * 64, img[:-1]):
        with pytest.raises(cilium_amd.PolicyError):
            b.import_tables(bad)
    b.import_tables(img)
    b.set_connections(w.conns)
    assert b.tables_digest == a.tables_digest and b.tables_compiled == 0


def test_import_refuses_inconsistent_image():
    """a well-framed image whose layout tag or offsets do not fit
    this build is refused (not read out of bounds)."""
    import struct
    import cilium_amd
    w = _workload()
    a = cilium_amd.Engine(-1)
    a.update_policy(w.policy)
    a.set_connections(w.conns)
    img = bytearray(a.export_tables())
    b = cilium_amd.Engine(-1)
    other_abi = bytearray(img)
    other_abi[8] ^= 1  # [magic | layout tag | form | px | policy source | HTTP rule sets ...]
    with pytest.raises(cilium_amd.PolicyError, match="layout"):
        b.import_tables(bytes(other_abi))
    (srclen,) = struct.unpack_from("<Q", img, 32)
    at = 40 + srclen
    (nrs,) = struct.unpack_from("<Q", img, at)
    assert nrs >= 1
    bad = bytearray(img)
    struct.pack_into("<I", bad, at + 8 + 4, 0xFFFFFFF0)  # rule set 0's image_len
    with pytest.raises(cilium_amd.PolicyError, match="inconsistent"):
        b.import_tables(bytes(bad))
    b.import_tables(bytes(img))
    b.set_connections(w.conns)
    assert b.tables_digest == a.tables_digest


def test_connection_outside_image_compiles_locally():
    """A rank whose connections need a rule set the exporter never compiled
    compiles just that one (same tables as compiling everything locally)."""
    import numpy as np
    import cilium_amd
    w = _workload()
    a = cilium_amd.Engine(-1)
    a.update_policy(w.policy)
    a.set_connections(w.conns[:1])
    b = cilium_amd.Engine(-1)
    b.import_tables(a.export_tables())
    b.set_connections(w.conns)
    c = cilium_amd.Engine(-1)
    c.update_policy(w.policy)
    c.set_connections(w.conns)
    assert b.tables_compiled > 0
    assert np.array_equal(np.array(sorted(b.stats().items())), np.array(sorted(c.stats().items())))


def test_large_nfa_tables_travel():
    """Rule sets with large NFAs (sparse follow rows, past 1,024 positions) ship
    in the exported image like any other table: the importer compiles nothing
    and installs byte-identical tables."""
    import sys
    import cilium_amd
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    import numpy as np
    import test_gpu_large_nfa as L
    from test_gpu_http import wl_from_reqs
    pol = L._policy(L.PATS[1])
    w = wl_from_reqs([b"x"] * 4, pol, L.CONNS, np.arange(4, dtype=np.uint32))
    a = cilium_amd.Engine(-1)
    a.update_policy(pol)
    a.set_connections(w.conns)
    assert a.stats()["http_nfas"] == 1 and a.stats()["nfa_pool_bytes"] > 100_000
    b = cilium_amd.Engine(-1)
    b.import_tables(a.export_tables())
    b.set_connections(w.conns)
    assert b.tables_compiled == 0 and b.tables_digest == a.tables_digest
