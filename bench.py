"""Benchmark: L7 verdicts/s + scanned GB/s (HBM roofline fraction) on MI355X.

One step = one l7g_classify pass over one batch of synthetic requests that are
already resident in HBM, plus the per-step RCCL all-reduce of the per-rule hit
counters when N > 1.

Default workload: cfg5 (BASELINE.json configs[4], the largest single-GPU
config and the one the "1/2/4/8 GPUs" metric names): 100M mixed requests per
GPU -- 50 % HTTP (cfg2's 64 rules), 30 % Kafka (cfg3's ~1k rules), 20 %
memcached text + binary -- built from a 2M-request unique stream.

Multi-GPU (N > 1, one process per GPU): every rank generates the SAME unique
stream (same seed, same policy), rank 0 compiles the policy for the node's
connections and broadcasts the compiled tables over RCCL (the other ranks
install them without compiling: l7g_tables_import), and the stream is sharded by connection (whole connections per rank,
each protocol's bytes balanced over ranks: cilium_amd/dist.py).  Each rank
tiles its shard up to the per-GPU request count (weak scaling), classifies it
every step and all-reduces the counters.  Every rank checks every verdict of
its last step against the oracle's verdicts for its shard; the mismatch count
is summed over ranks.

--workload picks another BASELINE.json config:
  cfg1  1 rule GET /public/.*            1M HTTP requests
  cfg2  64 HTTP rules                    1M HTTP requests
  cfg3  ~1k PortRuleKafka rules          1M Kafka requests
  cfg4  10k HTTP rules, 512 identities   10M HTTP requests (1M unique, tiled)
  cfg5  mixed HTTP/Kafka/memcached       100M requests (2M unique, tiled; default)

Besides the device-resident rate (`value`) the line reports:
  * roofline   -- the dominant kernel's algorithmic bytes / its device time
                  (HIP events around each launch, on the launch stream);
  * kernels    -- the same per kernel of the step;
  * e2e        -- pinned host arena -> H2D -> classify -> D2H, the unique
                  shard in 8 chunks on 2 streams (PCIe-inclusive; never `value`);
  * cpu_baseline -- the oracle (C restatement) on the host: all cores the
                  process may use, and one core, with nproc and the CPU model;
  * streams    -- the same unique requests regrouped into connection streams
                  (each connection's requests in order, cut into runs of 64:
                  what one proxylib OnData hands over) and decided through
                  l7g_classify_streams: device framing (a wave per HTTP /
                  memcached-text stream, a lane per Kafka / binary one) then
                  classification of every frame slot; frame-only ms, total ms,
                  bytes the framers read, parity of every frame vs the oracle;
  * latency    -- per-request latency of the drop-in paths (p50/p90/p99 us):
                  one request per l7g_classify_host call (the Envoy adapter's
                  Allowed()), requests through the asynchronous batcher
                  (l7g_batcher, 8 submitting threads at a fixed offered rate)
                  and proxylib OnData with one memcached request per call
                  (tests/native/latency_main.cc), next to the oracle deciding
                  one request per call on one core.

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

# workload -> (default requests per GPU, default unique requests, description)
WORKLOADS = {
    "cfg1": (1_000_000, 1_000_000, "cfg1: 1 HTTP rule {Method: GET, Path: /public/.*}, 256B-2KB HTTP/1.1 requests"),
    "cfg2": (1_000_000, 1_000_000, "cfg2: 64 HTTP rules (Method/Path/Host regex + literal X-Token), "
                                   "256B-2KB HTTP/1.1 requests"),
    "cfg3": (1_000_000, 1_000_000, "cfg3: Kafka produce/fetch/metadata stream, 1002 PortRuleKafka rules over 1k topics"),
    "cfg4": (10_000_000, 1_000_000, "cfg4: 10k HTTP rules across 512 remote identities (~20-rule groups), "
                                    "256B-2KB HTTP/1.1 requests"),
    "cfg5": (100_000_000, 2_000_000, "cfg5: mixed 50% HTTP (cfg2 rules) / 30% Kafka (cfg3 rules) / 20% memcached "
                                     "text+binary"),
}
KERNEL_NAMES = {"partition": "partition_kernel", "http": "http_classify_kernel",
                "kafka": "kafka_classify_kernel", "memcache": "memcache_classify_kernel"}


def make_workload(gen, name, n):
    cfg = int(name[3:])
    if cfg in (1, 2):
        return gen.http_workload(cfg, n)
    if cfg == 3:
        return gen.kafka_workload(n)
    if cfg == 4:
        return gen.cfg4_workload(n)
    return gen.mixed_workload(n)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_info():
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except AttributeError:
        usable = os.cpu_count() or 1
    # the process's CPU share: a cgroup quota caps what the affinity mask shows
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
            if path.endswith("cpu.max") and parts and parts[0] != "max":
                quota = int(parts[0]) / int(parts[1])
            elif path.endswith("quota_us") and parts and int(parts[0]) > 0:
                with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                    quota = int(parts[0]) / int(f.read())
        except (OSError, ValueError, IndexError):
            continue
        if quota:
            break
    share = max(1, min(usable, int(quota))) if quota else usable
    return {"nproc": os.cpu_count(), "usable_cores": share, "affinity_cores": usable, "cgroup_cpu_quota": quota,
            "model": model}


def e2e_pipeline(torch, eng, w, dev, nchunks=8, reps=3):
    """Pinned host arena -> H2D -> classify -> D2H for the unique shard, cut
    into nchunks request ranges alternating over two streams (the copies of
    one chunk overlap the kernels of the other).  Returns (seconds per pass,
    bytes moved per pass)."""
    n = w.n
    bounds = np.linspace(0, n, nchunks + 1).astype(np.int64)
    h_arena = torch.from_numpy(np.ascontiguousarray(w.arena)).pin_memory()
    offs = w.offsets.astype(np.int64)
    ends = offs + w.lengths.astype(np.int64)
    rel = np.empty(n, np.int64)
    spans = []
    for c in range(nchunks):
        a, b = bounds[c], bounds[c + 1]
        lo = int(offs[a:b].min()) if b > a else 0
        hi = int(ends[a:b].max()) if b > a else 0
        rel[a:b] = offs[a:b] - lo
        spans.append((a, b, lo, hi))
    h_off = torch.from_numpy(rel).pin_memory()
    h_len = torch.from_numpy(w.lengths.view(np.int32)).pin_memory()
    h_cid = torch.from_numpy(w.conn_ids.view(np.int32)).pin_memory()
    h_v = torch.empty(n, dtype=torch.uint8).pin_memory()
    h_r = torch.empty(n, dtype=torch.int32).pin_memory()
    h_c = torch.empty(n, dtype=torch.int32).pin_memory()
    max_bytes = max(hi - lo for _, _, lo, hi in spans) + 64
    max_req = int(max(b - a for a, b, _, _ in spans))
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    bufs = [dict(arena=torch.empty(max_bytes, dtype=torch.uint8, device=dev),
                 off=torch.empty(max_req, dtype=torch.int64, device=dev),
                 len=torch.empty(max_req, dtype=torch.int32, device=dev),
                 cid=torch.empty(max_req, dtype=torch.int32, device=dev),
                 v=torch.empty(max_req, dtype=torch.uint8, device=dev),
                 r=torch.empty(max_req, dtype=torch.int32, device=dev),
                 c=torch.empty(max_req, dtype=torch.int32, device=dev)) for _ in range(2)]
    done = [torch.cuda.Event(), torch.cuda.Event()]

    def one_pass():
        for c, (a, b, lo, hi) in enumerate(spans):
            k = c & 1
            s, B = streams[k], bufs[k]
            m = int(b - a)
            with torch.cuda.stream(s):
                s.wait_event(done[k])  # buffer set k: previous chunk's D2H finished
                B["arena"][:hi - lo].copy_(h_arena[lo:hi], non_blocking=True)
                B["off"][:m].copy_(h_off[a:b], non_blocking=True)
                B["len"][:m].copy_(h_len[a:b], non_blocking=True)
                B["cid"][:m].copy_(h_cid[a:b], non_blocking=True)
                eng.classify_device(B["arena"].data_ptr(), hi - lo, B["off"].data_ptr(), B["len"].data_ptr(),
                                    B["cid"].data_ptr(), m, B["v"].data_ptr(), B["r"].data_ptr(), B["c"].data_ptr(),
                                    stream=s.cuda_stream)
                h_v[a:b].copy_(B["v"][:m], non_blocking=True)
                h_r[a:b].copy_(B["r"][:m], non_blocking=True)
                h_c[a:b].copy_(B["c"][:m], non_blocking=True)
                done[k].record(s)
        torch.cuda.synchronize(dev)

    one_pass()  # warm-up (allocations, first-touch)
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        one_pass()
        ts.append(time.perf_counter() - t0)
    moved = sum(hi - lo for _, _, lo, hi in spans) + n * (16 + 9)
    return float(np.median(ts)), moved, (h_v.numpy().copy(), h_r.numpy().copy(), h_c.numpy().view(np.uint32).copy())


def streams_leg(torch, eng, gen, refpy, w, dev, threads, run=64, reps=10):
    """w's requests regrouped into connection streams (each connection's
    requests in order, cut into runs of `run`), framed and classified on the
    device by l7g_classify_streams; every frame's verdict / rule / consumed
    checked against the oracle on the same frame."""
    order = np.argsort(w.conn_ids, kind="stable")
    cid = w.conn_ids[order]
    offs = w.offsets[order].astype(np.int64)
    lens = w.lengths[order].astype(np.int64)
    cuts = np.flatnonzero(np.diff(cid)) + 1
    bounds = []
    for a, b in zip(np.r_[0, cuts], np.r_[cuts, len(cid)]):
        bounds.extend((k, min(k + run, b)) for k in range(a, b, run))
    buf = np.ascontiguousarray(w.arena)
    pieces, s_len, s_conn = [], [], []
    for a, b in bounds:
        pieces.extend(buf[offs[k]:offs[k] + lens[k]] for k in range(a, b))
        s_len.append(int(lens[a:b].sum()))
        s_conn.append(int(cid[a]))
    arena = np.concatenate(pieces)
    s_len = np.array(s_len, np.uint32)
    s_off = np.r_[0, np.cumsum(s_len[:-1], dtype=np.int64)].astype(np.uint64)
    s_conn = np.array(s_conn, np.uint32)
    ns, mf = len(bounds), run
    T = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    d_arena, d_soff, d_slen, d_sconn = T(arena), T(s_off.view(np.int64)), T(s_len.view(np.int32)), T(s_conn.view(np.int32))
    slots = ns * mf
    fo = torch.zeros(slots, dtype=torch.int64, device=dev)
    fl = torch.zeros(slots, dtype=torch.int32, device=dev)
    fc = torch.zeros(slots, dtype=torch.int32, device=dev)
    nf = torch.zeros(ns, dtype=torch.int32, device=dev)
    v = torch.zeros(slots, dtype=torch.uint8, device=dev)
    r = torch.zeros(slots, dtype=torch.int32, device=dev)
    c = torch.zeros(slots, dtype=torch.int32, device=dev)
    args = [d_arena.data_ptr(), arena.nbytes, d_soff.data_ptr(), d_slen.data_ptr(), d_sconn.data_ptr(), ns, mf,
            fo.data_ptr(), fl.data_ptr(), fc.data_ptr(), nf.data_ptr()]
    st = torch.cuda.current_stream()

    def timeit(f):
        f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(st)
        for _ in range(reps):
            f()
        e1.record(st)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    t_frame = timeit(lambda: eng.classify_streams_device(*args, stream=st.cuda_stream))
    t_all = timeit(lambda: eng.classify_streams_device(*args, v.data_ptr(), r.data_ptr(), c.data_ptr(),
                                                       stream=st.cuda_stream))
    nfr = nf.cpu().numpy()
    sel = np.concatenate([np.arange(s * mf, s * mf + nfr[s]) for s in range(ns)])
    fo_h = fo.cpu().numpy().view(np.uint64)[sel]
    fl_h = fl.cpu().numpy().view(np.uint32)[sel]
    fc_h = fc.cpu().numpy().view(np.uint32)[sel]
    ref = refpy.Policy(w.policy).classify(w.conns, arena, fo_h, fl_h, fc_h, threads)
    got = (v.cpu().numpy()[sel], r.cpu().numpy()[sel], c.cpu().numpy().view(np.uint32)[sel])
    mism = int(((got[0] != ref[0]) | (got[1] != ref[1]) | (got[2] != ref[2])).sum())
    # bytes the framers read: every byte of an HTTP / memcached-text / r2d2
    # stream (windows; bodies framed by length are not read), 16 B per frame of
    # a Kafka / memcached-binary / cassandra stream (the size field's chunk)
    proto = w.conns["proto"][s_conn]
    flags = w.conns["flags"][s_conn] & 3
    first = arena[s_off.astype(np.int64)]
    text = (proto == gen.PROTO_HTTP) | (proto == gen.PROTO_R2D2) | (
        (proto == gen.PROTO_MEMCACHE) & ((flags == 1) | ((flags == 0) & (first < 0x80))))
    read = int(s_len[text].astype(np.int64).sum()) + 16 * int(nfr[~text].sum())
    return {"streams": ns, "requests_per_stream_max": mf, "stream_bytes": int(arena.nbytes),
            "frames": int(nfr.sum()), "requests": w.n, "frame_ms": round(t_frame, 4),
            "frame_and_classify_ms": round(t_all, 4), "framer_bytes_read": read,
            "framer_read_gbps": round(read / (t_frame / 1e3) / 1e9, 1),
            "verdicts_per_s": round(int(nfr.sum()) / (t_all / 1e3), 1), "mismatches": mism,
            "note": "each connection's requests in order, cut into runs of 64 (one OnData buffer each); "
                    "l7g_classify_streams: framing, then every frame slot classified"}


def latency_leg(gen, refpy, iters=2000):
    """Drop-in path latency (rank 0, N = 1): tests/native/bin/latency_main on
    cfg2's HTTP requests and memcached text requests, and the oracle deciding
    the same requests one call at a time on one core."""
    import subprocess
    exe = os.path.join(ROOT, "tests", "native", "bin", "latency_main")
    if not os.path.exists(exe):
        return {"error": "tests/native/bin/latency_main not built"}
    h = gen.http_workload(2, 512)
    mreqs = [r for r in gen.memcache_requests(4000, 5) if r[0] < 0x80 and r.endswith(b"\r\n")][:512]
    mcp = gen.mc_policy()
    pol = {"policies": h.policy["policies"] + [dict(mcp["policies"][0], name="mc-lat")]}
    c0 = h.conns[0]
    hreqs = [bytes(h.arena[int(o):int(o) + int(n)]) for o, n in zip(h.offsets, h.lengths)]
    lines = [json.dumps(pol), f"{int(c0['policy'])} {int(c0['port'])} {int(c0['ingress'])} {int(c0['src_id'])} "
                              f"{int(c0['dst_id'])}", f"mc mc-lat {gen.MC_PORT} 3005"]
    lines += [r.hex() for r in hreqs] + ["--"] + [r.hex() for r in mreqs]
    try:
        r = subprocess.run([exe, str(iters)], input="\n".join(lines) + "\n", capture_output=True, text=True,
                           timeout=180)
        out = json.loads(r.stdout) if r.returncode == 0 else {"error": f"rc {r.returncode}: {r.stderr[-300:]}"}
    except Exception as e:  # the latency leg never fails the bench line
        out = {"error": repr(e)}
    # the oracle, one request per call, one core (ctypes call overhead included)
    P = refpy.Policy(pol)
    conns = np.concatenate([h.conns[:1], gen.make_conns(1, 1, gen.MC_PORT, True, gen.PROTO_MEMCACHE, [3005])])
    conns["flags"][1] = 1

    def one_by_one(reqs, cid):
        ts = []
        for q in reqs * max(1, iters // len(reqs)):
            a = np.frombuffer(q, np.uint8)
            t0 = time.perf_counter()
            P.classify(conns, a, np.zeros(1, np.uint64), np.array([len(q)], np.uint32), np.array([cid], np.uint32), 1)
            ts.append((time.perf_counter() - t0) * 1e6)
        ts.sort()
        return {"n": len(ts), "p50_us": ts[len(ts) // 2], "p99_us": ts[int(0.99 * (len(ts) - 1))]}
    out["oracle_one_core"] = {"http": one_by_one(hreqs, 0), "memcached": one_by_one(mreqs, 1),
                              "note": "refpy.Policy.classify with n=1 per call (ctypes overhead included)"}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="cfg5", choices=sorted(WORKLOADS))
    ap.add_argument("--requests", type=int, default=0, help="requests per GPU (weak scaling); 0 = workload default")
    ap.add_argument("--unique", type=int, default=0, help="unique requests generated (tiled up to --requests)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--no-streams", action="store_true")
    ap.add_argument("--cpu-threads", type=int, default=0, help="oracle threads (0 = every usable core)")
    ap.add_argument("--profile-steps", type=int, default=3, help="extra steps with per-kernel HIP events")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # Rehearsal of the N-rank path on a one-GPU box (tests/test_gpu_dist_bench.py):
    # L7G_DIST_BACKEND=gloo with L7G_DIST_ONE_DEVICE=1 puts every rank on cuda:0
    # (RCCL refuses two ranks on one device).  The driver's runs set neither.
    backend = os.environ.get("L7G_DIST_BACKEND", "nccl")
    if os.environ.get("L7G_DIST_ONE_DEVICE") == "1":
        local = 0

    import torch
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from cilium_amd import Engine, gen
    from cilium_amd import dist as l7dist

    dflt_n, dflt_u, wdesc = WORKLOADS[args.workload]
    want = args.requests or dflt_n
    uniq = args.unique or dflt_u
    t0 = time.time()
    # the same stream (and policy) on every rank: fixed per-config seed
    full = make_workload(gen, args.workload, uniq)
    if world > 1:
        _, shards = l7dist.shard_by_connection(full.conn_ids, full.lengths, len(full.conns), world,
                                               full.conns["proto"])
        w = gen.select(full, shards[rank], name=f"{full.name}[rank {rank}/{world}]")
    else:
        w = full
    nu = w.n
    tiles = max(1, want // max(nu, 1))
    offs, lens, cids = gen.tile_offsets(w, tiles)
    n = len(offs)
    pbytes = gen.protocol_bytes(w)
    log(f"[rank {rank}] {args.workload}: {full.n} unique requests generated, shard {nu} "
        f"({w.arena.nbytes / 1e9:.2f} GB) x {tiles} = {n} requests in {time.time() - t0:.1f}s")

    eng = Engine(local)
    # the policy arrives at rank 0 (the NPDS client), which compiles it for the
    # node's connections and broadcasts the compiled tables over RCCL; the other
    # ranks install them without compiling
    t_c = time.time()
    if dist is not None:
        l7dist.broadcast_tables(eng, dist, device=dev, policy=full.policy if rank == 0 else None,
                                conns=full.conns if rank == 0 else None)
    else:
        eng.update_policy(full.policy)
    eng.set_connections(w.conns)
    compile_s, compiled = time.time() - t_c, eng.tables_compiled
    other_compiled = 0
    if dist is not None:  # rule sets the ranks > 0 compiled themselves (0: all installed from rank 0's image)
        oc = torch.tensor([compiled if rank else 0], dtype=torch.int64, device=dev)
        dist.all_reduce(oc)
        other_compiled = int(oc.item())
    nrules = eng.nrules

    d_arena = torch.from_numpy(np.ascontiguousarray(w.arena)).to(dev)
    if tiles > 1:
        d_arena = d_arena.repeat(tiles)  # device-side replication of the unique shard
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
        # The counters kernel adds into the array it is given: one GPU accumulates
        # straight into the job's totals; with N GPUs each step's counters are
        # all-reduced first (the one collective on the data path).
        if dist is not None:
            step_counters.zero_()
        if i is not None:
            ev[i][0].record(stream)
        eng.classify_device(*ptrs, n, *outs, counters_ptr=(step_counters if dist is not None else totals).data_ptr(),
                            stream=stream.cuda_stream)
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

    # per-kernel device time: extra steps with HIP events around every launch
    stage_ms = {k: 0.0 for k in Engine.STAGES}
    if args.profile_steps > 0:
        eng.profile(True)
        acc = []
        for _ in range(args.profile_steps):
            eng.classify_device(*ptrs, n, *outs, stream=stream.cuda_stream)
            acc.append(eng.profile_last())
        eng.profile(False)
        stage_ms = {k: float(np.mean([a[k] for a in acc])) for k in Engine.STAGES}
    torch.cuda.synchronize()

    # parity of the last step on this rank's shard: every verdict, rule id and
    # consumed length against the oracle (test infrastructure, run after timing)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import refpy  # parity oracle: the checker and the CPU baseline, never the product path
    cinfo = cpu_info()
    threads = args.cpu_threads or cinfo["usable_cores"]  # every core of the process's CPU share
    verdict = d_v.cpu().numpy()
    rule = d_r.cpu().numpy()
    consumed = d_c.cpu().numpy().view(np.uint32)
    pol = refpy.Policy(full.policy)
    t1 = time.perf_counter()
    rv, rr, rc = pol.classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids, threads)
    cpu_all_s = time.perf_counter() - t1
    mism = 0
    for j in range(tiles):
        sl = slice(j * nu, (j + 1) * nu)
        mism += int(((verdict[sl] != rv) | (rule[sl] != rr) | (consumed[sl] != rc)).sum())
    if mism:
        log(f"[rank {rank}] PARITY FAILURE: {mism} of {n} requests differ from the oracle")

    # e2e: host arena in pinned memory, PCIe both ways, chunked on two streams
    e2e = None
    if not args.no_e2e:
        t_e2e, moved, eout = e2e_pipeline(torch, eng, w, dev)
        e2e_mism = int(((eout[0] != rv) | (eout[1] != rr) | (eout[2] != rc)).sum())
        e2e = {"s": t_e2e, "requests": nu, "bytes": moved, "mismatches": e2e_mism}

    # ---- aggregate over ranks
    if dist is not None:
        t = torch.tensor([elapsed, kernel_ms] + [stage_ms[k] for k in Engine.STAGES] +
                         [e2e["s"] if e2e else 0.0], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        vals = t.tolist()
        elapsed, kernel_ms = vals[0], vals[1]
        stage_ms = dict(zip(Engine.STAGES, vals[2:6]))
        if e2e:
            e2e["s"] = vals[6]
        cnt = torch.tensor([mism, n, nu, e2e["mismatches"] if e2e else 0, e2e["bytes"] if e2e else 0],
                           dtype=torch.int64, device=dev)
        dist.all_reduce(cnt)
        mism, checked, e2e_reqs, e2e_mism, e2e_bytes = [int(x) for x in cnt.tolist()]
        if e2e:
            e2e.update(requests=e2e_reqs, mismatches=e2e_mism, bytes=e2e_bytes)
    else:
        checked = n

    # CPU baseline (rank 0 at N = 1): the parity run above on every usable
    # core, plus one core on a bounded sample
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        m1 = min(nu, 300_000)
        sub = w.subset(np.arange(m1))
        t2 = time.perf_counter()
        refpy.Policy(w.policy).classify(sub.conns, sub.arena, sub.offsets, sub.lengths, sub.conn_ids, 1)
        cpu_1_s = time.perf_counter() - t2
        cpu = {"value": round(nu / cpu_all_s, 1), "unit": "verdicts/s", "cores": threads, "kind": "port",
               "sample": f"the {nu} unique requests of the {args.workload} arena ({w.arena.nbytes / 1e9:.2f} GB), one "
                         f"pass of the oracle/ C restatement on {threads} threads ({cpu_all_s:.2f} s wall); single "
                         f"core: the first {m1} requests ({cpu_1_s:.2f} s)",
               "scanned_gbps": round(float(w.lengths.astype(np.int64).sum()) / cpu_all_s / 1e9, 3),
               "single_core_verdicts_per_s": round(m1 / cpu_1_s, 1),
               "nproc": cinfo["nproc"], "usable_cores": cinfo["usable_cores"], "affinity_cores": cinfo["affinity_cores"],
               "cgroup_cpu_quota": cinfo["cgroup_cpu_quota"], "cpu_model": cinfo["model"]}

    latency = None
    if rank == 0 and world == 1 and not args.no_latency:
        latency = latency_leg(gen, refpy)
    streams = None
    if rank == 0 and world == 1 and not args.no_streams:
        try:
            streams = streams_leg(torch, eng, gen, refpy, w, dev, threads)
        except Exception as e:  # the streams leg never fails the bench line
            streams = {"error": repr(e)}

    if rank != 0:
        if dist is not None:
            dist.destroy_process_group()
        return

    total_requests = n * world * args.steps
    verdicts_per_s = total_requests / elapsed
    # algorithmic bytes per launch per GPU: payload + 25 B per request
    alg = {k: (pbytes[k]["payload"] + 25 * pbytes[k]["requests"]) * tiles for k in ("http", "kafka", "memcache")}
    n_other = pbytes["kafka"]["requests"] + pbytes["memcache"]["requests"]
    alg["partition"] = (8 * nu + 4 * n_other) * tiles if stage_ms["partition"] > 0 else 0
    step_alg = sum(alg[k] for k in ("http", "kafka", "memcache"))
    kernels = {}
    for k in Engine.STAGES:
        if stage_ms[k] > 0:
            g = alg[k] / (stage_ms[k] / 1e3) / 1e9
            kernels[k] = {"kernel": KERNEL_NAMES[k], "ms": round(stage_ms[k], 4), "algorithmic_bytes": alg[k],
                          "achieved_gbps": round(g, 1), "frac": round(g / HBM_PEAK_GBPS, 4)}
    dom = max((k for k in kernels if k != "partition"), key=lambda k: kernels[k]["ms"], default=None)
    traffic = None
    tpath = os.path.join(ROOT, "profiles", f"traffic_{args.workload}.json")
    # the PMC passes behind the file ran the workload's default size on one GPU
    measured_shape = world == 1 and args.requests in (0, dflt_n) and args.unique in (0, dflt_u)
    if dom and measured_shape and os.path.exists(tpath):
        try:
            with open(tpath) as f:
                tj = json.load(f)
            traffic = tj.get("kernels", {}).get(KERNEL_NAMES[dom], {}).get("hbm_bytes_per_launch")
            if traffic is None and len(kernels) == 1:
                traffic = tj.get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    if dom:
        achieved = alg[dom] / (stage_ms[dom] / 1e3) / 1e9
        roofline = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                    "frac": round(achieved / HBM_PEAK_GBPS, 4), "traffic": traffic, "kernel": KERNEL_NAMES[dom],
                    "kernel_ms": round(stage_ms[dom], 4), "algorithmic_bytes_per_launch": alg[dom]}
    else:
        roofline = None
    step_gbps = step_alg / (kernel_ms / 1e3) / 1e9
    hist = np.bincount(verdict, minlength=5)
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
                   "requests_per_gpu": n, "unique_requests": full.n, "unique_per_gpu": nu,
                   "global_requests_per_step": n * world,
                   "mean_request_bytes": round(float(w.lengths.mean()), 1),
                   "protocol_mix": {k: v["requests"] for k, v in pbytes.items()},
                   "parallelism": f"dp{world}" + (" (connection-sharded stream) + " +
                                                  ("RCCL" if backend == "nccl" else backend) + " counter all-reduce"
                                                  if world > 1 else "")},
        "tables": {"rank0_compile_s": round(compile_s, 3), "rank0_rulesets_compiled": compiled if rank == 0 else None,
                   "rulesets_compiled_by_other_ranks": other_compiled},
        "scanned_gbps": round(step_alg * world * args.steps / elapsed / 1e9, 2),
        "roofline": roofline,
        "step_roofline": {"algorithmic_bytes_per_launch": step_alg, "kernel_ms": round(kernel_ms, 4),
                          "achieved_gbps": round(step_gbps, 1), "frac": round(step_gbps / HBM_PEAK_GBPS, 4),
                          "note": "all kernels of one l7g_classify call, one HIP event pair on the stream"},
        "kernels": kernels,
        "cpu_baseline": cpu,
        "algorithmic_bytes_note": "per request len_i + 16 + 9 (SURVEY §8(d)); memcached counts only the bytes its "
                                  "parser must inspect (the command line, or the 24-byte header + extras + key; a "
                                  "storage command's data block is framed by length and never read), which lowers "
                                  "its frac against the len_i + 25 definition",
        "latency": latency,
        "streams": streams,
        "e2e": None if e2e is None else {
            "verdicts_per_s": round(e2e["requests"] / e2e["s"], 1), "ms_per_pass": round(e2e["s"] * 1e3, 3),
            "requests_per_pass": e2e["requests"], "pcie_gbps": round(e2e["bytes"] / e2e["s"] / 1e9, 2),
            "mismatches": e2e["mismatches"],
            "mode": "unique shard per GPU from pinned host memory: H2D arena + metadata, classify, D2H verdicts; "
                    "8 chunks alternating over 2 streams"},
        "parity": {"checked": checked, "mismatches": mism, "bit_exact": mism == 0,
                   "scope": "every request of the last step on every rank vs the oracle"},
        "verdict_hist_last_step_rank0": hist.tolist(),
        "counter_totals": {"allow_hits": int(tot[:nrules].sum()), "verdicts": tot[nrules:nrules + 5].tolist()},
    }
    print(json.dumps(line), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
