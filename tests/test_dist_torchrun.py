"""`torchrun --nproc-per-node 2` over gloo on CPU: bench.py's multi-GPU
sharding and counter path (tests/dist_worker.py), checked against the
unsharded stream."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world", [2, 3])
def test_torchrun_sharded_counters(tmp_path, world):
    out = tmp_path / "res.json"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "dist_worker.py"), "--out", str(out)]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=500, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.load(open(out))
    assert res["compiled_by_other_ranks"] == 0  # ranks > 0 installed rank 0's compiled tables
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import bench
    import refpy
    from cilium_amd import gen
    full = bench.make_workload(gen, "cfg5", 20000)
    v, rr, _ = refpy.Policy(full.policy).classify(full.conns, full.arena, full.offsets, full.lengths, full.conn_ids)
    nr = res["nrules"]
    want = np.zeros(nr + 8, np.int64)
    want[nr:nr + 5] = np.bincount(v, minlength=5)[:5]
    want[:nr] = np.bincount(rr[rr >= 0], minlength=nr)[:nr]
    assert res["counters"] == want.tolist()  # all-reduced shards == the whole stream
    per = np.array(res["per_rank"])
    assert per[:, 0].sum() == full.n and (per[:, 0] > 0).all()  # every request on exactly one rank
    for k in (2, 3, 4):  # each protocol's bytes balanced over ranks
        if per[:, k].sum():
            assert per[:, k].max() / (per[:, k].sum() / world) < 1.35
