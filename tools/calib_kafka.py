"""Kafka traffic calibration (GPU box; measurement tool).  cfg5's Kafka
requests (one unique tile, in the Kafka kernel's list order: kind / length
class, longest first) are read once each by tools/calib/kafka_traffic.hip in
three access patterns, and then classified by the product Kafka kernel on the
same arena.  Run under rocprofv3 --pmc <counter> --kernel-trace: the
per-dispatch FETCH_SIZE (or raw TCC counters) of each calib kernel against the
printed byte count fixes the counter's scale for that access pattern.
usage: python tools/calib_kafka.py [unique_requests]"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)
from cilium_amd import Engine, gen  # noqa: E402
from cilium_amd._lib import PROTO_KAFKA  # noqa: E402

LIB = os.path.join(HERE, "calib", "libcalib.so")


def build():
    src = os.path.join(HERE, "calib", "kafka_traffic.hip")
    if not os.path.exists(LIB) or os.path.getmtime(LIB) < os.path.getmtime(src):
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "--offload-arch=gfx950", "-shared", "-fPIC", src, "-o", LIB],
                       check=True)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
    build()
    lib = ctypes.CDLL(LIB)
    lib.calib_read.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p]
    w = gen.mixed_workload(n)
    kafka = np.nonzero(w.conns["proto"][w.conn_ids] == PROTO_KAFKA)[0]
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(w.arena).to(dev)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    s = torch.cuda.current_stream()
    # stream order (a lane's neighbours read the lines next to its own), and by
    # length, longest first (the Kafka kernel's class order taken to the limit:
    # no two lanes of a wave near each other in the arena)
    for order in ("stream", "len"):
        keep = kafka if order == "stream" else kafka[np.argsort(-w.lengths[kafka].astype(np.int64), kind="stable")]
        off, ln = w.offsets[keep], w.lengths[keep]
        chunks = (((off + ln + 15) & ~np.uint64(15)) - (off & ~np.uint64(15))) // 16
        nbytes = int(chunks.sum()) * 16
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_len = torch.from_numpy(ln.view(np.int32)).to(dev)
        print(f"[{order}] kafka requests {len(keep)}  request bytes {int(ln.sum())}  chunk bytes read per calib "
              f"launch {nbytes}  arena {w.arena.nbytes}", flush=True)
        for mode, name in ((0, "lane16"), (1, "lane64"), (2, "wave")):
            for _ in range(2):
                rc = lib.calib_read(d_arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(keep), mode,
                                    sink.data_ptr(), ctypes.c_void_p(s.cuda_stream))
                assert rc == 0, rc
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(s)
            lib.calib_read(d_arena.data_ptr(), d_off.data_ptr(), d_len.data_ptr(), len(keep), mode, sink.data_ptr(),
                           ctypes.c_void_p(s.cuda_stream))
            e1.record(s)
            torch.cuda.synchronize()
            ms = e0.elapsed_time(e1)
            print(f"[{order}] calib {name}: {ms:.3f} ms  {nbytes / ms / 1e6:.1f} GB/s", flush=True)
    keep = kafka
    d_len = torch.from_numpy(w.lengths[keep].view(np.int32)).to(dev)
    # the product Kafka kernel on the same requests (its own order: partition lists)
    eng = Engine(0)
    k = gen.Workload("cfg5-kafka", w.arena, w.offsets[keep], w.lengths[keep], w.conn_ids[keep], w.conns, w.policy, {})
    eng.update_policy(k.policy)
    eng.set_connections(k.conns)
    d_o2 = torch.from_numpy(k.offsets.view(np.int64)).to(dev)
    outs = [torch.empty(k.n, dtype=t, device=dev) for t in (torch.uint8, torch.int32, torch.int32)]
    for _ in range(3):
        eng.classify_device(d_arena.data_ptr(), d_arena.numel(), d_o2.data_ptr(), d_len.data_ptr(),
                            torch.from_numpy(k.conn_ids.view(np.int32)).to(dev).data_ptr(), k.n,
                            *[t.data_ptr() for t in outs], stream=s.cuda_stream)
    torch.cuda.synchronize()
    print(f"kafka kernel: {k.n} requests, {int(k.lengths.sum())} bytes", flush=True)


if __name__ == "__main__":
    main()
