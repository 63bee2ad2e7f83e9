"""One memcached request per l7g_classify_host call (the OnData shape) in a loop,
for rocprofv3 --kernel-trace --stats (GPU box): the kernels' own duration."""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, gen  # noqa: E402


def main():
    mreqs = [r for r in gen.memcache_requests(4000, 5) if r[0] < 0x80 and r.endswith(b"\r\n")][:512]
    pol = gen.mc_policy()
    conns = gen.make_conns(1, 0, gen.MC_PORT, True, gen.PROTO_MEMCACHE, [3005])
    conns["flags"][0] = 1
    eng = Engine(0)
    eng.update_policy(pol)
    eng.set_connections(conns)
    ts = []
    for i in range(3000):
        q = np.frombuffer(mreqs[i % len(mreqs)], np.uint8)
        t0 = time.perf_counter()
        eng.classify(q, np.zeros(1, np.uint64), np.array([len(q)], np.uint32), np.zeros(1, np.uint32))
        ts.append((time.perf_counter() - t0) * 1e6)
    ts = sorted(ts[200:])
    print(f"classify_host n=1 memcached: p50 {ts[len(ts) // 2]:.1f} us  p99 {ts[int(len(ts) * 0.99)]:.1f} us (Python call included)")


if __name__ == "__main__":
    main()
