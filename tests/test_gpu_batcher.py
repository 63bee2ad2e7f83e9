"""l7g_batcher on the GPU (tests/native/batcher_parity_main.cc): requests
submitted from 8 threads come back with exactly the verdict, rule id and
consumed count one synchronous l7g_classify_host call over the same requests
gives -- through small batches (packed, read in place over PCIe) and through
large ones (lanes copied as separate pieces, entries closed up), for HTTP and
for Kafka (the partitioned path)."""
import json
import os
import subprocess

import numpy as np
import pytest

from cilium_amd import gen

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "bin", "batcher_parity_main")


def _stdin(w):
    reqs = [bytes(w.arena[int(o):int(o) + int(n)]) for o, n in zip(w.offsets, w.lengths)]
    lines = [json.dumps(w.policy), np.ascontiguousarray(w.conns).tobytes().hex()]
    lines += [f"{int(c)} {q.hex()}" for c, q in zip(w.conn_ids, reqs)]
    return "\n".join(lines) + "\n"


def _run(w, max_n, wait_us, threads=8):
    assert os.path.exists(EXE), "built by __graft_entry__.build() / cilium_amd.build.build_test_natives()"
    r = subprocess.run([EXE, str(max_n), str(wait_us), str(threads)], input=_stdin(w), capture_output=True,
                       text=True, timeout=100)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout)


@pytest.mark.parametrize("max_n,wait_us", [(8, 50), (256, 100), (4096, 200)])
def test_batcher_http_matches_sync(max_n, wait_us):
    w = gen.http_workload(2, 12000)
    d = _run(w, max_n, wait_us)
    assert d["n"] == 12000 and d["requests"] == 12000, d
    assert d["calls_not_once"] == 0 and d["mismatches"] == 0, d
    assert 0 < d["allowed"] < d["n"], d  # both verdicts exercised
    if max_n == 4096:
        assert d["max_batch"] > 256, d  # the copied (not packed) path ran


def test_batcher_kafka_matches_sync():
    w = gen.kafka_workload(6000)
    d = _run(w, 1024, 200)
    assert d["n"] == 6000 and d["mismatches"] == 0 and d["calls_not_once"] == 0, d
