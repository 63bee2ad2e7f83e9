"""Per-rule allow hits and per-verdict totals (l7g_classify `counters`,
kernels/counters.hip) against the oracle's histogram of its own verdicts:
a batch whose length is not a multiple of the kernel's 4-entry groups, output
arrays that are only 4-byte aligned (the rule loads fall back to dwords), and
hot rules (one rule allowing most requests: the lanes of a wave sharing a bin
are added as one count)."""
import numpy as np
import pytest
import torch

from cilium_amd import gen

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("cfg,n,shift", [(1, 300_001, 0), (2, 200_003, 1), (1, 7, 1)])
def test_counters_match_oracle_histogram(engine, oracle, cfg, n, shift):
    w = gen.http_workload(cfg, n)
    ref = oracle.classify_workload(w, 8)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(w.arena).to(dev)
    d_off = torch.from_numpy(w.offsets.view(np.int64)).to(dev)
    d_len = torch.from_numpy(w.lengths.view(np.int32)).to(dev)
    d_cid = torch.from_numpy(w.conn_ids.view(np.int32)).to(dev)
    # rule[] at a 4-byte (not 16-byte) aligned address when shift = 1
    d_v = torch.empty(w.n, dtype=torch.uint8, device=dev)
    d_rbuf = torch.empty(w.n + 4, dtype=torch.int32, device=dev)
    d_r = d_rbuf[shift:shift + w.n]
    d_c = torch.empty(w.n, dtype=torch.int32, device=dev)
    nr = engine.nrules
    cnt = torch.zeros(nr + 8, dtype=torch.int64, device=dev)
    for _ in range(2):  # accumulated over two calls
        engine.classify_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(),
                               d_cid.data_ptr(), w.n, d_v.data_ptr(), d_r.data_ptr(), d_c.data_ptr(),
                               counters_ptr=cnt.data_ptr())
    torch.cuda.synchronize()
    assert (d_v.cpu().numpy() == ref[0]).all() and (d_r.cpu().numpy() == ref[1]).all()
    want = np.zeros(nr + 8, np.int64)
    allow = ref[0] == 1
    np.add.at(want, ref[1][allow], 2)
    for v in range(5):
        want[nr + v] = 2 * int((ref[0] == v).sum())
    got = cnt.cpu().numpy()
    assert (got == want).all(), (np.nonzero(got != want)[0][:8], got[:8], want[:8])
