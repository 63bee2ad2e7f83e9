"""Benchmark: L7 verdicts/s + scanned GB/s (HBM roofline fraction) on MI355X.

One step = one classification pass over one batch of synthetic requests that
are already resident in HBM (default: BASELINE.json configs[1] = cfg2: 64 HTTP
rules over Method/Path/Host regexes + literal X-Token header, 256 B-2 KB
HTTP/1.1 requests, 1M requests per GPU), plus the per-step RCCL all-reduce of
the per-rule hit counters when N > 1.  Weak scaling: every rank classifies its
own shard (request batches are independent; no payload crosses GPUs).

--workload picks another BASELINE.json config:
  cfg1  1 rule GET /public/.*            1M HTTP requests
  cfg2  64 HTTP rules (default)          1M HTTP requests
  cfg3  ~1k PortRuleKafka rules          1M Kafka requests
  cfg4  10k HTTP rules, 512 identities   10M HTTP requests (1M unique, tiled)
  cfg5  mixed HTTP/Kafka/memcached       100M requests (2M unique, tiled)
Tiled workloads replicate the unique arena on the device; every copy is
checked against the oracle's verdicts of the unique part.

Usage:  python bench.py [--gpus N --steps K --warmup W --workload cfgX]
        (N > 1: python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...)
Rank 0 prints one JSON line.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E peak (/opt/skills/guides/MI355X_MICROARCH.md)
METRIC = "L7 verdicts/sec + scanned GB/s (HBM roofline frac), 1/2/4/8 MI355X"

# workload -> (default requests per GPU, default unique requests, description, kernel(s) timed)
WORKLOADS = {
    "cfg1": (1_000_000, 1_000_000, "cfg1: 1 HTTP rule {Method: GET, Path: /public/.*}, 256B-2KB HTTP/1.1 requests",
             "http_classify_kernel"),
    "cfg2": (1_000_000, 1_000_000, "cfg2: 64 HTTP rules (Method/Path/Host regex + literal X-Token), "
                                   "256B-2KB HTTP/1.1 requests", "http_classify_kernel"),
    "cfg3": (1_000_000, 1_000_000, "cfg3: Kafka produce/fetch/metadata stream, 1002 PortRuleKafka rules over 1k topics",
             "partition_kernel (length classes) + kafka_classify_kernel"),
    "cfg4": (10_000_000, 1_000_000, "cfg4: 10k HTTP rules across 512 remote identities (~20-rule groups), "
                                    "256B-2KB HTTP/1.1 requests", "http_classify_kernel"),
    "cfg5": (100_000_000, 2_000_000, "cfg5: mixed 50% HTTP (cfg2 rules) / 30% Kafka (cfg3 rules) / 20% memcached "
                                     "text+binary", "partition + http + kafka + memcache kernels (4 launches)"),
}


def make_workload(gen, name, n, seed):
    cfg = int(name[3:])
    if cfg in (1, 2):
        return gen.http_workload(cfg, n, seed=seed)
    if cfg == 3:
        return gen.kafka_workload(n, seed=seed)
    if cfg == 4:
        return gen.cfg4_workload(n, seed=seed)
    return gen.mixed_workload(n, seed=seed)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg2", choices=sorted(WORKLOADS))
    ap.add_argument("--requests", type=int, default=0, help="requests per GPU (weak scaling); 0 = workload default")
    ap.add_argument("--unique", type=int, default=0, help="unique requests generated (tiled up to --requests)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("nccl", device_id=dev)

    from cilium_amd import Engine, gen
    from cilium_amd import dist as l7dist

    dflt_n, dflt_u, wdesc, kname = WORKLOADS[args.workload]
    want = args.requests or dflt_n
    uniq = min(args.unique or dflt_u, want)
    tiles = max(1, want // uniq)
    t0 = time.time()
    w = make_workload(gen, args.workload, uniq, gen.SEED_BASE + int(args.workload[3:]) + 7919 * rank)
    nu = w.n
    offs, lens, cids = gen.tile_offsets(w, tiles)
    n = len(offs)
    log(f"[rank {rank}] {args.workload}: generated {nu} unique requests ({w.arena.nbytes / 1e9:.2f} GB) x {tiles} "
        f"= {n} requests in {time.time() - t0:.1f}s")

    eng = Engine(local)
    # the policy arrives at rank 0 (NPDS) and is broadcast to every rank over RCCL
    policy = l7dist.broadcast_policy(w.policy, dist, device=dev) if dist is not None else w.policy
    eng.update_policy(policy)
    eng.set_connections(w.conns)
    nrules = eng.nrules

    d_arena = torch.from_numpy(w.arena).to(dev)
    if tiles > 1:
        d_arena = d_arena.repeat(tiles)  # device-side replication of the unique arena
    d_off = torch.from_numpy(offs.view(np.int64)).to(dev)
    d_len = torch.from_numpy(lens.view(np.int32)).to(dev)
    d_cid = torch.from_numpy(cids.view(np.int32)).to(dev)
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_r = torch.empty(n, dtype=torch.int32, device=dev)
    d_c = torch.empty(n, dtype=torch.int32, device=dev)
    step_counters = torch.zeros(nrules + 8, dtype=torch.int64, device=dev)
    totals = torch.zeros(nrules + 8, dtype=torch.int64, device=dev)
    stream = torch.cuda.current_stream()
    ptrs = [d_arena.data_ptr(), d_arena.numel()] + [t.data_ptr() for t in (d_off, d_len, d_cid)]
    outs = [t.data_ptr() for t in (d_v, d_r, d_c)]

    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    def step(i=None):
        step_counters.zero_()
        if i is not None:
            ev[i][0].record(stream)
        eng.classify_device(*ptrs, n, *outs, counters_ptr=step_counters.data_ptr(), stream=stream.cuda_stream)
        if i is not None:
            ev[i][1].record(stream)
        if dist is not None:
            l7dist.allreduce_counters(step_counters, dist)  # RCCL over xGMI: per-rule hit counters
        totals.add_(step_counters)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    if dist is not None:
        t = torch.tensor([elapsed, kernel_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kernel_ms = float(t[0]), float(t[1])

    total_requests = n * world * args.steps
    verdicts_per_s = total_requests / elapsed
    alg_bytes = w.algorithmic_bytes() * tiles  # per launch, per GPU
    scanned_gbps = alg_bytes * world * args.steps / elapsed / 1e9
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    # ---- parity of the last step on this rank's shard + CPU baseline (oracle, N = 1 only)
    verdict = d_v.cpu().numpy()
    rule = d_r.cpu().numpy()
    consumed = d_c.cpu().numpy().view(np.uint32)
    parity = None
    cpu = None
    if world == 1 and not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        import refpy  # parity oracle: the checker and the CPU baseline, never the product path
        try:
            cores = len(os.sched_getaffinity(0))
        except AttributeError:
            cores = os.cpu_count() or 1
        cores = args.cpu_threads or min(16, cores)
        pol = refpy.Policy(w.policy)
        t1 = time.perf_counter()
        rv, rr, rc = pol.classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids, cores)
        cpu_s = time.perf_counter() - t1
        cpu = {"value": round(nu / cpu_s, 1), "unit": "verdicts/s", "cores": cores, "kind": "port",
               "sample": f"the {nu} unique requests of the {args.workload} arena, one pass, oracle/ C restatement "
                         f"on {cores} threads ({cpu_s:.2f} s wall, {w.arena.nbytes / 1e9:.2f} GB)",
               "scanned_gbps": round(w.lengths.astype(np.int64).sum() / cpu_s / 1e9, 3)}
        rv, rr, rc = (np.tile(a, tiles) for a in (rv, rr, rc))
        mism = int(((verdict != rv) | (rule != rr) | (consumed != rc)).sum())
        parity = {"checked": n, "mismatches": mism, "bit_exact": mism == 0}
        if mism:
            log(f"PARITY FAILURE: {mism} of {n} requests differ from the oracle")

    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    if os.path.exists(tpath):
        try:
            with open(tpath) as f:
                traffic = json.load(f).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None

    hist = np.bincount(verdict, minlength=5)
    if args.workload == "cfg5":
        line_extra = {"protocol_mix": {"http": int((w.conns["proto"][w.conn_ids] == 1).sum()),
                                       "kafka": int((w.conns["proto"][w.conn_ids] == 2).sum()),
                                       "memcache": int((w.conns["proto"][w.conn_ids] == 3).sum())}}
    else:
        line_extra = {}
    tot = totals.cpu().numpy()
    line = {
        "metric": METRIC,
        "value": round(verdicts_per_s, 1),
        "unit": "verdicts/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / args.steps * 1e3, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": f"{wdesc}, {n} requests per GPU",
                   "requests_per_gpu": n, "unique_requests": nu, "global_requests_per_step": n * world,
                   "mean_request_bytes": round(float(w.lengths.mean()), 1),
                   "parallelism": f"dp{world}" + (" + RCCL counter all-reduce" if world > 1 else "")},
        "scanned_gbps": round(scanned_gbps, 2),
        "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic,
                     "kernel": kname, "kernel_ms": round(kernel_ms, 4),
                     "algorithmic_bytes_per_launch": alg_bytes},
        "cpu_baseline": cpu,
        "parity": parity,
        "verdict_hist_last_step": hist.tolist(),
        "counter_totals": {"allow_hits": int(tot[:nrules].sum()), "verdicts": tot[nrules:nrules + 5].tolist()},
        **line_extra,
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
