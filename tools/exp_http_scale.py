"""HTTP kernel at the bench's scale (GPU box): cfg5's 1M unique HTTP requests
packed, then the same requests cut before their long X-Pad line ("heads":
the same request lines and header lines up to the token, then the empty
line), each tiled on the device to N requests (the bench's replication), and
the HTTP kernel time per 1M requests (HIP events, l7g profile).  The gap
between the two is what streaming the pad bytes costs beyond the head parse.
usage: python tools/exp_http_scale.py [tiles]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cilium_amd import Engine, gen  # noqa: E402
from cilium_amd._lib import PROTO_HTTP  # noqa: E402


def run(eng, name, reqs, conn_ids, conns, policy, tiles):
    arena, offs, lens = gen.pack(reqs)
    w = gen.Workload(name, arena, offs, lens, conn_ids, conns, policy)
    o, l, c = gen.tile_offsets(w, tiles)
    dev = torch.device("cuda", 0)
    d_a = torch.from_numpy(arena).to(dev).repeat(tiles)
    d_o = torch.from_numpy(o.view(np.int64)).to(dev)
    d_l = torch.from_numpy(l.view(np.int32)).to(dev)
    d_c = torch.from_numpy(c.view(np.int32)).to(dev)
    n = len(o)
    outs = [torch.empty(n, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
    eng.update_policy(policy)
    eng.set_connections(conns)
    eng.profile(True)
    s = torch.cuda.current_stream()
    ms = []
    for it in range(8):
        eng.classify_device(d_a.data_ptr(), d_a.numel(), d_o.data_ptr(), d_l.data_ptr(), d_c.data_ptr(), n,
                            *[t.data_ptr() for t in outs], stream=s.cuda_stream)
        p = eng.profile_last()
        if it >= 2:
            ms.append(p["http"])
    torch.cuda.synchronize()
    k = float(np.median(ms))
    gb = (float(lens.astype(np.int64).sum()) + 25.0 * len(lens)) * tiles / 1e9
    print(f"{name:8s} n={n} mean_len={lens.mean():.0f}  http {k:.3f} ms  {k / n * 1e6:.4f} ms/1M  "
          f"{gb / (k / 1e3):.0f} GB/s  verdicts {np.bincount(outs[0][:len(lens)].cpu().numpy(), minlength=5).tolist()}",
          flush=True)
    del d_a, d_o, d_l, d_c, outs
    torch.cuda.empty_cache()


def main():
    tiles = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    w = gen.mixed_workload(2_000_000)
    keep = np.nonzero(w.conns["proto"][w.conn_ids] == PROTO_HTTP)[0]
    reqs = [bytes(w.arena[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in keep]
    heads = [r[: r.index(b"X-Pad: ")] + b"\r\n" for r in reqs]
    eng = Engine(0)
    for name, rr in (("full", reqs), ("heads", heads), ("full", reqs)):
        run(eng, name, rr, w.conn_ids[keep], w.conns, w.policy, tiles)


if __name__ == "__main__":
    main()
