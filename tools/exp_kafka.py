"""Kafka kernel experiment (GPU box): cfg3 at N requests through the product
library and variant builds side by side (libl7gpu_<name>.so, built with
`python -m cilium_amd.build --variant NAME -DX`).  Prints per-variant kernel
time (HIP events around the launch, median of 10) and parity vs the oracle.

usage: python tools/exp_kafka.py N variant...   ("prod" = libl7gpu.so)
"""
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def main():
    import torch
    import refpy
    from cilium_amd import Engine, gen
    n = int(sys.argv[1])
    names = sys.argv[2:] or ["prod"]
    wl = os.environ.get("EXP_WORKLOAD", "cfg3")
    t0 = time.time()
    if wl.startswith("cfg3"):
        w = gen.kafka_workload(n)
        if wl != "cfg3":  # cfg3produce / cfg3fetch / cfg3other: one kind's requests of the cfg3 stream
            kinds = np.array([int(w.arena[int(o) + 4]) << 8 | int(w.arena[int(o) + 5]) for o in w.offsets])
            want = {"cfg3produce": kinds == 0, "cfg3fetch": kinds == 1, "cfg3other": kinds > 1}[wl]
            w = gen.select(w, np.nonzero(want)[0], wl)
            n = w.n
    elif wl in ("produni", "prodcnt"):  # produce requests of one fixed structure (divergence probe)
        rng = np.random.default_rng(7)
        topics = gen.kafka_topics()
        reqs = []
        for i in range(n):
            tps = []
            for t in range(2):
                k = 2 if t == 0 else 3
                ln = [288] * k if wl == "produni" else [int(rng.integers(64, 513)) for _ in range(k)]
                msgs = [gen.k_message(rng.integers(0, 256, size=L, dtype=np.uint8).tobytes(),
                                      key=None if i % 2 else b"k%d" % i, version=i % 3) for L in ln]
                tps.append((topics[int(rng.integers(0, 1000))], [(0, msgs)]))
            reqs.append(gen.k_produce(i % 3, i, "client-%02d" % (i % 16), tps))
        arena, offs, lens = gen.pack(reqs)
        conn_ids = rng.integers(0, 256, size=n).astype(np.uint32)
        conns = gen.make_conns(256, 0, 9092, True, gen.PROTO_KAFKA, 2000 + np.arange(256))
        w = gen.Workload(wl, arena, offs, lens, conn_ids, conns, gen.cfg3_policy())
    elif wl == "mc":  # memcached alone (cfg5's memcached stream)
        w = gen.memcache_workload(n)
    else:
        w = gen.mixed_workload(n)
    print(f"{wl}: {n} requests, {w.arena.nbytes / 1e6:.1f} MB, generated in {time.time() - t0:.1f}s", flush=True)
    ref = refpy.classify_workload(w, 16)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(np.ascontiguousarray(a)).to(dev) for a in
         (w.arena, w.offsets.view(np.int64), w.lengths.view(np.int32), w.conn_ids.view(np.int32))]
    outs = [torch.empty(n, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
    s = torch.cuda.current_stream()
    # algorithmic bytes of the Kafka kernel: the Kafka requests' bytes + 25 per
    # Kafka request (not the whole mixed workload's)
    kb = gen.protocol_bytes(w)["kafka"]
    gb = (kb["payload"] + 25 * kb["requests"]) / 1e9
    for name in names:
        path = os.path.join(ROOT, "cilium_amd", "libl7gpu.so" if name == "prod" else f"libl7gpu_{name}.so")
        eng = Engine(0, lib_path=path)
        eng.update_policy(w.policy)
        eng.set_connections(w.conns)
        eng.profile(True)
        ms = []
        for it in range(13):
            eng.classify_device(d[0].data_ptr(), d[0].numel(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n,
                                *[o.data_ptr() for o in outs], stream=s.cuda_stream)
            p = eng.profile_last()
            if it >= 3:
                ms.append(p)
        torch.cuda.synchronize()
        got = (outs[0].cpu().numpy(), outs[1].cpu().numpy(), outs[2].cpu().numpy().view(np.uint32))
        mism = int(((got[0] != ref[0]) | (got[1] != ref[1]) | (got[2] != ref[2])).sum())
        med = {k: float(np.median([m[k] for m in ms])) for k in ms[0] if ms[0][k] > 0}
        kms = med.get("kafka", 0.0)
        print(f"{name:12s} " + " ".join(f"{k}={v:.3f}ms" for k, v in med.items()) +
              (f"  kafka {gb / (kms / 1e3):.0f} GB/s frac {gb / (kms / 1e3) / 8000:.3f}" if kms else "") +
              f"  mismatches={mism}", flush=True)
        ph = eng.kafka_phase_times()
        if ph is not None:
            tot = float(ph[:6].sum()) or 1.0
            print("   phases: " + " ".join(f"{k}={ph[i] / tot:.3f}" for i, k in
                                           enumerate(["setup", "walk", "-", "crc", "-", "redo+out"])) +
                  f"  groups={ph[6] / 13:.0f} redone-lanes={ph[7] / 13:.0f}"
                  f" cycles/group={tot / max(ph[6], 1):.0f}", flush=True)
        eng.close()


if __name__ == "__main__":
    main()
