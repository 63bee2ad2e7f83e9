"""bench.py's N-rank path with device verdicts, rehearsed on a one-GPU box:
`torchrun --nproc-per-node 2 bench.py --gpus 2` with both ranks on cuda:0 over
gloo (RCCL refuses two ranks on one device; the driver's 8-GPU runs use RCCL,
one rank per GPU).  What runs is the product path of every rank: rank 0
compiles and broadcasts the compiled tables, rank 1 installs them without
compiling, each rank classifies its connection shard on the device, the per-rule
counters are all-reduced every step, and the timing is the max over ranks.
Every rank checks its last step against the oracle."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.timeout(420)
def test_bench_two_ranks_one_device():
    warmup, steps = 1, 3
    cmd = [sys.executable, "-u", "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "cfg5", "--requests", "2000000",
           "--unique", "100000", "--steps", str(steps), "--warmup", str(warmup), "--no-cpu-baseline", "--no-e2e",
           "--no-latency", "--no-streams", "--profile-steps", "1", "--cpu-threads", "4"]
    env = dict(os.environ, L7G_DIST_BACKEND="gloo", L7G_DIST_ONE_DEVICE="1", OMP_NUM_THREADS="4")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=400, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["scaling"] == "weak"
    assert d["parity"]["mismatches"] == 0 and d["parity"]["bit_exact"]
    checked = d["parity"]["checked"]  # both ranks' requests of the last step
    assert checked > d["config"]["requests_per_gpu"]
    assert d["tables"]["rulesets_compiled_by_other_ranks"] == 0
    # counters: every request of every step on both ranks, summed by the all-reduce
    assert sum(d["counter_totals"]["verdicts"]) == (warmup + steps) * checked
    assert d["value"] > 0 and d["ms_per_step"] > 0
    assert "gloo counter all-reduce" in d["config"]["parallelism"]
    assert d["roofline"]["traffic"] is None  # the PMC traffic files hold the one-GPU default size only
    print(lines[0])
