"""bench.py's N > 1 path on CPU (gloo), launched by torchrun from
tests/test_dist_torchrun.py: the same stream on every rank (bench.make_workload,
fixed seed), rank 0's compiled tables broadcast (installed, not compiled, by the other
ranks), the stream sharded by connection with
each protocol's bytes balanced (cilium_amd/dist.py, what bench.py calls), rank
0's tables compiled by the product compiler (host-only engine), per-rank
counters all-reduced, parity counts summed, timings MAX-reduced.  The device
verdicts are stood in for by the oracle here (no GPU): this checks the
exchange, the sharding and the counter path, not the kernels."""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--unique", type=int, default=20000)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    world, rank = int(os.environ["WORLD_SIZE"]), int(os.environ["RANK"])
    dist.init_process_group("gloo")
    try:
        import bench
        import refpy
        import cilium_amd
        from cilium_amd import dist as l7dist, gen
        full = bench.make_workload(gen, "cfg5", args.unique)
        _, shards = l7dist.shard_by_connection(full.conn_ids, full.lengths, len(full.conns), world, full.conns["proto"])
        w = gen.select(full, shards[rank], name=f"{full.name}[rank {rank}/{world}]")
        eng = cilium_amd.Engine(-1)
        # rank 0 compiles, the others install its compiled tables (bench.py's path)
        image = l7dist.broadcast_tables(eng, dist, policy=full.policy if rank == 0 else None,
                                        conns=full.conns if rank == 0 else None)
        eng.set_connections(w.conns)
        policy = full.policy  # for the oracle, which stands in for the device verdicts
        compiled = torch.tensor([eng.tables_compiled if rank else 0], dtype=torch.int64)
        dist.all_reduce(compiled)
        nr = eng.nrules
        t0 = time.perf_counter()
        v, r, c = refpy.Policy(policy).classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids)
        elapsed = time.perf_counter() - t0
        # the counters l7g_classify would return for this rank's shard
        cnt = torch.zeros(nr + 8, dtype=torch.int64)
        cnt[nr:nr + 5] = torch.from_numpy(np.bincount(v, minlength=5)[:5].astype(np.int64))
        hit = r[r >= 0]
        cnt[:nr] = torch.from_numpy(np.bincount(hit, minlength=nr)[:nr].astype(np.int64))
        l7dist.allreduce_counters(cnt, dist)
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        pb = gen.protocol_bytes(w)
        tot = torch.tensor([w.n, int(w.lengths.astype(np.int64).sum())] + [int(pb[k]["payload"]) for k in ("http", "kafka", "memcache")],
                           dtype=torch.int64)
        per = [torch.zeros_like(tot) for _ in range(world)]
        dist.all_gather(per, tot)
        if rank == 0:
            json.dump({"world": world, "n_full": full.n, "counters": cnt.tolist(), "max_s": float(t.item()),
                       "per_rank": [p.tolist() for p in per], "nrules": nr,
                       "compiled_by_other_ranks": int(compiled.item()),
                       "stats": {k: v for k, v in eng.stats().items() if k.startswith(("http", "kafka", "mc"))}},
                      open(args.out, "w"))
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
