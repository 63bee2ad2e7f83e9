"""Kernel-time decomposition experiments for the HTTP classifier (GPU box).
Times l7g_classify on device-resident batches for several request/policy
variants and prints ms per 1M requests and achieved GB/s."""
import sys
import os
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, api, gen  # noqa: E402


def timeit(eng, w, steps=10):
    dev = torch.device("cuda", 0)
    d_a = torch.from_numpy(w.arena).to(dev)
    d_o = torch.from_numpy(w.offsets.view(np.int64)).to(dev)
    d_l = torch.from_numpy(w.lengths.view(np.int32)).to(dev)
    d_c = torch.from_numpy(w.conn_ids.view(np.int32)).to(dev)
    n = w.n
    d_v = torch.empty(n, dtype=torch.uint8, device=dev)
    d_r = torch.empty(n, dtype=torch.int32, device=dev)
    d_k = torch.empty(n, dtype=torch.int32, device=dev)
    eng.update_policy(w.policy)
    eng.set_connections(w.conns)
    eng.phase_times(reset=True)
    s = torch.cuda.current_stream()
    args = [d_a.data_ptr(), d_a.numel()] + [t.data_ptr() for t in (d_o, d_l, d_c)] + [n] + \
        [t.data_ptr() for t in (d_v, d_r, d_k)]
    for _ in range(3):
        eng.classify_device(*args, stream=s.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        eng.classify_device(*args, stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / steps
    gbps = w.algorithmic_bytes() / (ms / 1e3) / 1e9
    hist = np.bincount(d_v.cpu().numpy(), minlength=5).tolist()
    ph = eng.phase_times(reset=True)
    if ph is not None:
        eng.classify_device(*args, stream=s.cuda_stream)
        torch.cuda.synchronize()
        ph = eng.phase_times(reset=True).astype(np.float64)
        cyc = ph[:4].sum()
        hist = hist + [f"dma {ph[0]/cyc:.2f} parse {ph[1]/cyc:.2f} scan {ph[2]/cyc:.2f} other {ph[3]/cyc:.2f} "
                       f"rounds/tile {ph[4]/max(ph[6],1):.2f} scans/tile {ph[5]/max(ph[6],1):.1f} "
                       f"wave-cycles/tile {cyc/max(ph[6],1):.0f}"]
    return ms, gbps, hist


def variant(name, reqs, policy, nconns=1024):
    arena, offs, lens = gen.pack(reqs)
    rng = np.random.default_rng(1)
    conns = gen.make_conns(nconns, 0, 80, True, 1, 1000 + np.arange(nconns))
    return gen.Workload(name, arena, offs, lens, rng.integers(0, nconns, len(reqs)).astype(np.uint32), conns, policy)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000
    only = sys.argv[2].split(",") if len(sys.argv) > 2 else None  # variant letters a..e
    lib = os.environ.get("EXP_LIB")
    eng = Engine(0, lib_path=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cilium_amd", lib)) if lib else Engine(0)
    base = gen.http_requests(n, gen.SEED_BASE + 2)
    heads = [r[: r.index(b"X-Pad: ")] + b"\r\n" for r in base]
    allow_all = api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(80, [api.port_rule()])]))
    rows = [
        ("cfg2 full", variant("a", base, gen.cfg2_policy())),
        ("cfg1 policy, full", variant("b", base, gen.cfg1_policy())),
        ("no http rules, full", variant("c", base, allow_all)),
        ("cfg2 heads only", variant("d", heads, gen.cfg2_policy())),
        ("no rules heads only", variant("e", heads, allow_all)),
    ]
    # per-line cost: k unknown 20-byte header lines after a fixed request line
    for k, letter in ((0, "f"), (4, "g"), (8, "h")):
        reqs = [b"GET /abcdefghijklmnop HTTP/1.1\r\n" + b"X-Aaaa: 0123456789\r\n" * k + b"\r\n"] * n
        rows.append((f"no rules, {k} lines", variant(letter, reqs, allow_all)))
    reqs = [b"GET /abcdefghijklmnop HTTP/1.1\r\n" + b"Host: 0123456789abc\r\n" * 4 + b"\r\n"] * n
    rows.append(("cfg2 pol, 4 host lines", variant("i", reqs, gen.cfg2_policy())))
    for name, w in rows:
        if only and w.name not in only:
            continue
        ms, gbps, hist = timeit(eng, w)
        print(f"{name:24s} n={w.n} bytes={w.lengths.astype(np.int64).sum()/w.n:7.1f}/req  {ms:8.4f} ms  "
              f"{gbps:8.1f} GB/s  {ms / w.n * 1e6:7.4f} ms/1M  hist={hist}", flush=True)


if __name__ == "__main__":
    main()
