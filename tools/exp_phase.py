"""HTTP kernel phase split on cfg5's HTTP requests where they lie in the mixed
arena (GPU box; run with EXP_LIB=libl7gpu_timing.so for the phase cycles:
python -m cilium_amd.build --timing).  Prints ms per 1M requests and the
fraction of wave cycles in window DMA / parse / tile map + skips / other."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from cilium_amd import Engine, gen  # noqa: E402
from cilium_amd._lib import PROTO_HTTP  # noqa: E402
from exp_http import timeit  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    lib = os.environ.get("EXP_LIB")
    here = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    eng = Engine(0, lib_path=os.path.join(here, "cilium_amd", lib)) if lib else Engine(0)
    w = gen.mixed_workload(n)
    keep = np.nonzero(w.conns["proto"][w.conn_ids] == PROTO_HTTP)[0]
    g = gen.Workload("http-in-place", w.arena, w.offsets[keep], w.lengths[keep], w.conn_ids[keep], w.conns, w.policy, {})
    ms, gbps, hist = timeit(eng, g)
    print(f"cfg5 HTTP in place  n={g.n}  {ms:8.4f} ms  {gbps:8.1f} GB/s  {ms / g.n * 1e6:7.4f} ms/1M  {hist}", flush=True)
    reqs = [bytes(w.arena[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in keep[:1_000_000]]
    heads = [r[: r.index(b"X-Pad: ")] + b"\r\n" for r in reqs]
    for name, rr in (("cfg5 HTTP packed", reqs), ("cfg5 heads packed", heads)):
        arena, offs, lens = gen.pack(rr)
        h = gen.Workload(name, arena, offs, lens, w.conn_ids[keep[:len(rr)]], w.conns, w.policy, {})
        ms, gbps, hist = timeit(eng, h)
        print(f"{name:18s}  n={h.n}  {ms:8.4f} ms  {gbps:8.1f} GB/s  {ms / h.n * 1e6:7.4f} ms/1M  {hist}", flush=True)


if __name__ == "__main__":
    main()
