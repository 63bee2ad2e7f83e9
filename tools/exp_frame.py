"""Device framing throughput (GPU box): l7g_frame_streams and
l7g_classify_streams on connection streams built from a workload's requests
(one stream per connection, requests in order), next to l7g_classify on the
same frames with host-known offsets.  Prints ms and GB/s of stream bytes.

usage: python tools/exp_frame.py [http|kafka|memcache] [requests] [connections]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, gen  # noqa: E402


def main():
    kind = sys.argv[1] if len(sys.argv) > 1 else "http"
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 1_000_000
    nconns = int(sys.argv[3]) if len(sys.argv) > 3 else 16384
    w = {"http": lambda: gen.http_workload(2, n, nconns=nconns), "kafka": lambda: gen.kafka_workload(n, nconns=nconns),
         "memcache": lambda: gen.memcache_workload(n, nconns=nconns)}[kind]()
    order = np.argsort(w.conn_ids, kind="stable")
    cid = w.conn_ids[order]
    reqs = [bytes(w.arena[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in order]
    arena, offs, lens = gen.pack(reqs)
    conns_used, first = np.unique(cid, return_index=True)
    s_off = offs[first].astype(np.uint64)
    ends = np.append(first[1:], len(reqs))
    s_len = np.array([int(offs[e - 1]) + int(lens[e - 1]) - int(offs[b]) for b, e in zip(first, ends)], np.uint32)
    per = ends - first
    mf = int(per.max())
    lib = os.environ.get("L7G_LIB")
    eng = Engine(0, lib_path=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cilium_amd", f"libl7gpu_{lib}.so")) if lib else Engine(0)
    eng.update_policy(w.policy)
    eng.set_connections(w.conns)
    dev = torch.device("cuda", 0)
    T = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.itemsize == 4 else a).to(dev)  # noqa: E731
    d_arena, d_soff, d_slen, d_sconn = T(arena), T(s_off), T(s_len), T(conns_used.astype(np.uint32))
    ns = len(s_off)
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
    s = torch.cuda.current_stream()

    def timeit(f, steps=10):
        for _ in range(2):
            f()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(steps):
            f()
        e1.record(s)
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / steps

    eng.frame_phase_times(True)
    t_frame = timeit(lambda: eng.classify_streams_device(*args, stream=s.cuda_stream))
    ph = eng.frame_phase_times(True)
    if ph is not None and ph[4]:
        print(f"  text framer per stream: {ph[1] / ph[4]:.0f} cycles, window loads {ph[2] / ph[4]:.1f} "
              f"({ph[0] / max(ph[2], 1):.0f} cycles each, {ph[0] / max(ph[1], 1):.2f} of the time), frames {ph[3] / ph[4]:.1f}")
    t_both = timeit(lambda: eng.classify_streams_device(*args, v.data_ptr(), r.data_ptr(), c.data_ptr(),
                                                        stream=s.cuda_stream))
    got = int(nf.sum().item())
    # the same requests with host-known offsets (each handed its own bytes)
    d_off, d_len, d_cid = T(offs.astype(np.uint64)), T(lens.astype(np.uint32)), T(cid.astype(np.uint32))
    v2 = torch.zeros(len(reqs), dtype=torch.uint8, device=dev)
    r2 = torch.zeros(len(reqs), dtype=torch.int32, device=dev)
    c2 = torch.zeros(len(reqs), dtype=torch.int32, device=dev)
    t_plain = timeit(lambda: eng.classify_device(d_arena.data_ptr(), arena.nbytes, d_off.data_ptr(), d_len.data_ptr(),
                                                 d_cid.data_ptr(), len(reqs), v2.data_ptr(), r2.data_ptr(),
                                                 c2.data_ptr(), stream=s.cuda_stream))
    gb = arena.nbytes / 1e9
    print(f"{kind}: {len(reqs)} requests in {ns} streams (<= {mf} frames each), {gb:.3f} GB; frames found {got}")
    print(f"  frame_streams    {t_frame:8.3f} ms  {gb / t_frame * 1e3:7.1f} GB/s")
    print(f"  classify_streams {t_both:8.3f} ms  {gb / t_both * 1e3:7.1f} GB/s  (framing + classification over {slots} slots)")
    print(f"  classify (host-known offsets) {t_plain:8.3f} ms")


if __name__ == "__main__":
    main()
