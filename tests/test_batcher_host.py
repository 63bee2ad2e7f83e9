"""l7g_batcher's threading on the CPU (tests/native/batcher_stress.cc on a
host-only engine): lock-free submit from 8 threads into the pinned slots, two
flushers, every callback once and in each thread's submission order, flush,
re-entrant flush refused, backpressure once both flushers are busy and the open
slot is full."""
import json
import subprocess

import pytest

from cilium_amd import build as b


@pytest.mark.timeout(300)
def test_batcher_threads_order_flush_backpressure():
    exe = [x for x in b.build_test_natives() if x.endswith("batcher_stress")][0]
    r = subprocess.run([exe], capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr
    d = json.loads(r.stdout)
    assert d["bad"] == 0, d
    assert d["after_flush"] == d["expected"], d  # flush returned after every callback
    assert d["calls"] == d["expected"] + d["large_expected"], d
    assert d["flush_rc"] == 0 and d["reentrant_flush_rc"] == -1, d
    assert d["launches"] < d["expected"] // 8, d  # batched, not one launch per request
    assert d["large_calls"] == d["large_expected"], d  # byte-full slots (holes closed up): every callback once
    assert d["huge_rc"] == -2, d  # larger than a lane: refused
    assert d["slow_max"] == 4 and d["big_max"] == 65536, d  # the effective batch size, capped
    # both flushers blocked in callbacks: at most two sealed batches and one full open slot are taken
    assert d["refused"] > 0 and d["queued"] + d["refused"] == 5000, d
    assert 1024 <= d["queued"] <= 3 * 1024 and d["slow_answered"] == d["queued"], d
