"""Mixed-batch experiment (GPU box): the HTTP kernel's time on cfg5's HTTP
requests inside the mixed batch vs the same HTTP requests packed alone.
Run under rocprofv3 --kernel-trace --stats for per-kernel times."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, gen  # noqa: E402
from cilium_amd._lib import PROTO_HTTP  # noqa: E402


def run(eng, w, steps, tag):
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(x).to(dev) for x in (w.arena, w.offsets.view(np.int64), w.lengths.view(np.int32),
                                               w.conn_ids.view(np.int32))]
    n = w.n
    out = [torch.empty(n, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
    eng.update_policy(w.policy)
    eng.set_connections(w.conns)
    s = torch.cuda.current_stream()
    args = [d[0].data_ptr(), d[0].numel()] + [t.data_ptr() for t in d[1:]] + [n] + [t.data_ptr() for t in out]
    for _ in range(2):
        eng.classify_device(*args, stream=s.cuda_stream)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(s)
    for _ in range(steps):
        eng.classify_device(*args, stream=s.cuda_stream)
    e1.record(s)
    torch.cuda.synchronize()
    print(f"{tag:28s} n={n} {e0.elapsed_time(e1) / steps:8.3f} ms/step  stats={ {k: v for k, v in eng.stats().items() if 'hot' in k or 'cold' in k} }",
          flush=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 4_000_000
    lib = os.environ.get("EXP_LIB")
    eng = Engine(0, lib_path=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cilium_amd", lib)) if lib else Engine(0)
    w = gen.mixed_workload(n)
    run(eng, w, 5, "mixed")
    proto = w.conns["proto"][w.conn_ids]
    keep = np.nonzero(proto == PROTO_HTTP)[0]
    reqs = [bytes(w.arena[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in keep]
    arena, offs, lens = gen.pack(reqs)
    h = gen.Workload("http-only", arena, offs, lens, w.conn_ids[keep], w.conns, w.policy, {})
    run(eng, h, 5, "same HTTP requests, packed")
    # the HTTP requests where they lie in the mixed arena (gaps between them),
    # classified on their own: memory layout vs the mixed launch itself
    g = gen.Workload("http-in-place", w.arena, w.offsets[keep], w.lengths[keep], w.conn_ids[keep], w.conns, w.policy, {})
    run(eng, g, 5, "same HTTP requests, in place")
    # the same packed HTTP requests plus one memcached request: the partition
    # path (HTTP list) with contiguous tiles
    mc = np.nonzero(proto != PROTO_HTTP)[0][:1]
    reqs2 = reqs + [bytes(w.arena[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in mc]
    arena, offs, lens = gen.pack(reqs2)
    h2 = gen.Workload("http+1", arena, offs, lens, np.concatenate([w.conn_ids[keep], w.conn_ids[mc]]), w.conns, w.policy, {})
    run(eng, h2, 5, "packed HTTP + 1 other (list)")


if __name__ == "__main__":
    main()
