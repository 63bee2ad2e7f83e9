"""Debug: one large mixed batch through the product library vs the oracle,
mismatches per protocol and the unwritten (sentinel) outputs."""
import os, sys
import numpy as np
import torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
from cilium_amd import Engine, gen
import refpy

u = gen.mixed_workload(200_000)
ref_u = refpy.classify_workload(u, 8)
n = (1 << 20) + 4321
k = -(-n // u.n)
idx = np.tile(np.arange(u.n), k)[:n]
w = gen.Workload("t", u.arena, u.offsets[idx], u.lengths[idx], u.conn_ids[idx], u.conns, u.policy)
ref = tuple(np.concatenate([r] * k)[:n] for r in ref_u)
proto = w.conns["proto"][w.conn_ids]
for lib in sys.argv[1:] or ["libl7gpu.so"]:
    eng = Engine(0, lib_path=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "cilium_amd", lib))
    eng.update_policy(w.policy)
    eng.set_connections(w.conns)
    dev = torch.device("cuda", 0)
    d = [torch.from_numpy(x).to(dev) for x in (w.arena, w.offsets.view(np.int64), w.lengths.view(np.int32), w.conn_ids.view(np.int32))]
    for sname, s in (("default", torch.cuda.current_stream()), ("side", torch.cuda.Stream())):
        o = [torch.full((n,), 7, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
        with torch.cuda.stream(s):
            eng.classify_device(d[0].data_ptr(), d[0].numel(), d[1].data_ptr(), d[2].data_ptr(), d[3].data_ptr(), n,
                                *[t.data_ptr() for t in o], stream=s.cuda_stream)
        torch.cuda.synchronize()
        v, r, c = o[0].cpu().numpy(), o[1].cpu().numpy(), o[2].cpu().numpy().view(np.uint32)
        bad = (v != ref[0]) | (r != ref[1]) | (c != ref[2])
        print(lib, sname, "bad", int(bad.sum()), {int(p): int((bad & (proto == p)).sum()) for p in np.unique(proto)},
              "unwritten", int((v == 7).sum()), "bad idx", np.nonzero(bad)[0][:6], flush=True)
        if bad.any():
            i = np.nonzero(bad)[0][0]
            print("  first bad", i, "proto", int(proto[i]), "got", int(v[i]), int(r[i]), int(c[i]), "want", int(ref[0][i]), int(ref[1][i]), int(ref[2][i]))
    eng.close()
