"""Multi-GPU plumbing for the verdict path.

One process per GPU.  Requests are independent given their connection, so
the data path shards by connection with no collective; the two exchange
steps are
  * compiled tables: the policy set (cilium.NetworkPolicy list) arrives at
    rank 0 (the NPDS client, proxylib/proxylib/instance.go:168-219), which
    compiles it (regex -> DFA / NFA, Kafka topic views) for every connection
    of the node and broadcasts the compiled image (l7g_tables_export: the
    policy source plus every rule set's device bytes and the rule-list ->
    rule-set cache); the other ranks install it (l7g_tables_import) without
    compiling -- one compile per node, not one per GPU;
  * per-rule hit counters: one all-reduce(sum) of the (rules + 8) uint64
    counters per batch (the UpdateProxyStatistics feed,
    pkg/endpoint/endpoint.go:2207-2233).
`torch.distributed` with backend "nccl" is RCCL over xGMI on the MI355X box;
the same functions run over "gloo" on CPU tensors in the tests.
"""
import json

import numpy as np


def broadcast_policy(policy, dist, src=0, device=None):
    """Return the policy JSON bytes held by `src` on every rank.
    `policy` (dict / str / bytes) is only read on `src`."""
    import torch
    rank = dist.get_rank()
    if rank == src:
        b = policy if isinstance(policy, bytes) else (policy if isinstance(policy, str) else json.dumps(policy)).encode()
        n = torch.tensor([len(b)], dtype=torch.int64, device=device)
    else:
        b = None
        n = torch.zeros(1, dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def _broadcast_bytes(b, dist, src, device):
    """b (read on src only) on every rank; b is None on src -> None everywhere
    (the length word carries -1 and no payload follows)."""
    import torch
    rank = dist.get_rank()
    n = torch.tensor([(-1 if b is None else len(b)) if rank == src else 0], dtype=torch.int64, device=device)
    dist.broadcast(n, src)
    if int(n.item()) < 0:
        return None
    buf = torch.empty(int(n.item()), dtype=torch.uint8, device=device)
    if rank == src:
        buf.copy_(torch.frombuffer(bytearray(b), dtype=torch.uint8))
    dist.broadcast(buf, src)
    return bytes(buf.cpu().numpy().tobytes())


def broadcast_tables(engine, dist, src=0, device=None, policy=None, conns=None):
    """Rank `src` compiles (`policy` and the node's connection table `conns`,
    both read on `src` only) and broadcasts its compiled tables; every other
    rank installs them into `engine` without compiling.  Returns the image
    bytes.  Over RCCL (backend "nccl", device = the rank's GPU) on the box,
    gloo on CPU in the tests.

    A policy `src` refuses (PolicyError: the NPDS NACK) still completes the
    collective: `src` broadcasts "no image", every rank keeps the version it
    has (as the reference keeps the previous policy on a NACK,
    proxylib/proxylib/instance.go:168-219), the other ranks return None and
    `src` re-raises."""
    rank = dist.get_rank()
    err = None
    image = None
    if rank == src:
        try:
            if policy is not None:
                engine.update_policy(policy)
            if conns is not None:
                engine.set_connections(conns)
            image = engine.export_tables()
        except Exception as e:  # noqa: BLE001 -- re-raised below, after the collective
            err, image = e, None
    image = _broadcast_bytes(image, dist, src, device)
    if err is not None:
        raise err
    if rank != src and image is not None:
        engine.import_tables(image)
    return image


def allreduce_counters(counters, dist):
    """Sum per-rule hit counters (int64 tensor, rules + 8) over all ranks, in place."""
    dist.all_reduce(counters)
    return counters


def shard_by_connection(conn_ids, lengths, nconns, world, conn_proto=None):
    """Assign whole connections to ranks (a connection's stream stays on one
    GPU: framing state, reply queues, Kafka close-on-error) so that every rank
    gets an equal share of the payload bytes -- of each protocol separately
    when conn_proto (protocol per connection) is given, since an HTTP byte, a
    Kafka byte and a memcached byte do not cost the same device time.  Within
    a protocol, ranks own contiguous connection-id ranges.  Returns
    (owner[nconns], sorted request index array per rank)."""
    conn_ids = np.asarray(conn_ids, np.int64)
    per_conn = np.bincount(conn_ids, weights=np.asarray(lengths, np.float64), minlength=nconns)[:nconns]
    owner = np.zeros(nconns, np.int64)
    groups = [np.arange(nconns)] if conn_proto is None else \
        [np.nonzero(np.asarray(conn_proto) == p)[0] for p in np.unique(conn_proto)]
    for g in groups:
        if len(g) == 0:
            continue
        b = per_conn[g]
        cum = np.cumsum(b)
        total = cum[-1]
        # connection c goes to the rank whose byte range holds its midpoint
        mid = cum - b / 2
        o = np.minimum((mid * world // max(total, 1.0)).astype(np.int64), world - 1)
        owner[g] = np.maximum.accumulate(o)  # contiguous, non-decreasing ranges
    valid = conn_ids < nconns
    req_owner = np.where(valid, owner[np.minimum(conn_ids, max(nconns - 1, 0))], conn_ids % max(world, 1))
    return owner, [np.nonzero(req_owner == r)[0] for r in range(world)]
