"""Where a one-request HTTP call's device time goes (GPU box).

Runs l7g_classify (device-resident inputs) with n = 1 on the latency leg's
requests (cfg2 policy, hot rule set) and on a request that ends at once, and
prints the per-call device time (HIP events) and, with a -DL7G_PHASE_TIMING
build (L7G_LIB=...), the HTTP kernel's phase cycles per call."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, gen  # noqa: E402


def main():
    h = gen.http_workload(2, 512)
    eng = Engine(device=0)
    eng.update_policy(h.policy)
    eng.set_connections(h.conns)
    dev = torch.device("cuda", 0)
    s = torch.cuda.current_stream()
    cases = {"cfg2": [bytes(h.arena[int(o):int(o) + int(n)]) for o, n in zip(h.offsets[:200], h.lengths[:200])],
             "bad": [b"X\r\n\r\n"] * 200,
             "tiny": [b"GET / HTTP/1.1\r\nHost: a\r\n\r\n"] * 200}
    cid = torch.zeros(1, dtype=torch.int32, device=dev)
    d_v = torch.empty(1, dtype=torch.uint8, device=dev)
    d_r = torch.empty(1, dtype=torch.int32, device=dev)
    d_k = torch.empty(1, dtype=torch.int32, device=dev)
    d_o = torch.zeros(1, dtype=torch.int64, device=dev)
    for name, reqs in cases.items():
        ts, phs = [], []
        for q in reqs:
            a = torch.from_numpy(np.frombuffer(q + bytes(16), np.uint8).copy()).to(dev)
            d_l = torch.tensor([len(q)], dtype=torch.int32, device=dev)
            torch.cuda.synchronize()
            eng.phase_times(reset=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            eng.classify_device(a.data_ptr(), len(q), d_o.data_ptr(), d_l.data_ptr(), cid.data_ptr(), 1,
                                d_v.data_ptr(), d_r.data_ptr(), d_k.data_ptr(), stream=s.cuda_stream)
            e1.record(s)
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1) * 1e3)
            ph = eng.phase_times(reset=True)
            if ph is not None:
                phs.append(ph.astype(np.float64))
        ts.sort()
        line = f"{name}: len {np.mean([len(q) for q in reqs]):.0f} B, device p50 {ts[len(ts)//2]:.1f} us p10 {ts[len(ts)//10]:.1f}"
        if phs:
            m = np.mean(phs[5:], axis=0)
            line += (f" | cycles: stage {m[7]:.0f} map/emit {m[2]:.0f} dma {m[0]:.0f} parse {m[1]:.0f} other {m[3]:.0f}"
                     f" rounds {m[4]:.1f} scans {m[5]:.1f}")
            if m[13]:  # well-formed-head shortcut (lat_fast): scan, lines, walks (merge+end under 11 when it declines)
                line += (f" | lat_fast: load+masks {m[13]:.0f} block checks {m[9]:.0f} line parse {m[10]:.0f}"
                         f" slots {m[14]:.0f} walks {m[15]:.0f} merge {m[11]:.0f}")
            elif m[12]:  # latency kernel (one request per wave)
                line += (f" | latency kernel: fetch {m[8]:.0f} CR scan {m[9]:.0f} lines {m[10]:.0f}"
                         f" merge+end {m[11]:.0f}")
        print(line, flush=True)


if __name__ == "__main__":
    main()
