"""cfg4 at its configured size on the GPU (BASELINE.json configs[3]).

10,000 HTTP rules across 512 remote identities (~20-rule PortNetworkPolicyRule
groups with remote_policies), requests from connections uniform over the 512
identities plus 2 % unknown ones.  Checks, against the oracle:

  * every verdict, matched rule id and consumed length of 200k requests;
  * the device's per-rule hit counters (l7g_classify `counters`) against the
    oracle's rule-hit histogram -- rule ids run to ~10k, so most counters go
    through the kernel's global-atomic path (ids >= 1016), not the LDS one;
  * the per-verdict totals.

Reference semantics: envoy/cilium_network_policy.h:128-192 (PortNetworkPolicy
rule groups, remote sets), pkg/envoy/server.go:476-537.
"""
import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, DENY

from test_gpu_http import assert_same

pytestmark = pytest.mark.gpu

N = 200_000


@pytest.fixture(scope="module")
def cfg4():
    return gen.cfg4_workload(N)


def test_cfg4_full_size_parity_and_counters(engine, oracle, cfg4):
    import torch

    w = cfg4
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    nrules = engine.nrules
    assert nrules == 10_000
    st = engine.stats()
    assert st["http_rulesets"] >= 512
    dev = torch.device("cuda", 0)
    d_arena = torch.from_numpy(w.arena).to(dev)
    d_off = torch.from_numpy(w.offsets.view(np.int64)).to(dev)
    d_len = torch.from_numpy(w.lengths.view(np.int32)).to(dev)
    d_cid = torch.from_numpy(w.conn_ids.view(np.int32)).to(dev)
    d_v = torch.empty(w.n, dtype=torch.uint8, device=dev)
    d_r = torch.empty(w.n, dtype=torch.int32, device=dev)
    d_c = torch.empty(w.n, dtype=torch.int32, device=dev)
    counters = torch.zeros(nrules + 8, dtype=torch.int64, device=dev)
    s = torch.cuda.current_stream()
    engine.classify_device(d_arena.data_ptr(), d_arena.numel(), d_off.data_ptr(), d_len.data_ptr(), d_cid.data_ptr(),
                           w.n, d_v.data_ptr(), d_r.data_ptr(), d_c.data_ptr(), counters_ptr=counters.data_ptr(),
                           stream=s.cuda_stream)
    torch.cuda.synchronize()
    got = (d_v.cpu().numpy(), d_r.cpu().numpy(), d_c.cpu().numpy().view(np.uint32))
    ref = oracle.classify_workload(w, 16)
    assert_same(got, ref, w)
    v, r = ref[0], ref[1]
    assert (v == ALLOW).sum() > 200 and (v == DENY).mean() > 0.3
    cnt = counters.cpu().numpy()
    hits = np.bincount(r[(v == ALLOW) & (r >= 0)], minlength=nrules)[:nrules]
    assert hits[1016:].sum() > 0, "no rule id >= 1016 was hit: the global counter path is not covered"
    np.testing.assert_array_equal(cnt[:nrules], hits)
    np.testing.assert_array_equal(cnt[nrules:nrules + 5], np.bincount(v, minlength=5)[:5])


def _merge(a, b, seed=5):
    """a's and b's requests interleaved in one batch (b's policy appended, its
    connections after a's), as gen.mixed_workload merges its three streams."""
    pol = {"policies": [a.policy["policies"][0], dict(b.policy["policies"][0], name="10.0.0.2")]}
    conns = np.concatenate([a.conns, b.conns])
    conns["policy"][len(a.conns):] = 1
    offs = np.concatenate([a.offsets, b.offsets + np.uint64(len(a.arena))])
    lens = np.concatenate([a.lengths, b.lengths])
    cids = np.concatenate([a.conn_ids, b.conn_ids + np.uint32(len(a.conns))])
    perm = np.random.default_rng(seed).permutation(len(offs))
    buf = np.concatenate([a.arena, b.arena]).tobytes()
    arena, o2, l2 = gen.pack([buf[int(o):int(o) + int(n)] for o, n in zip(offs[perm], lens[perm])])
    return gen.Workload("merged", arena, o2, l2, cids[perm], conns, pol, {})


def test_grouped_path_in_a_mixed_batch(engine, oracle):
    """cfg4's HTTP requests among Kafka requests: the protocol split runs first
    and the grouped HTTP path sorts the partition's HTTP list by rule set."""
    w = _merge(gen.cfg4_workload(90_000, seed=41), gen.kafka_workload(30_000, seed=43))
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 16), w)


def test_grouped_path_big_images(engine, oracle):
    """Rule sets whose image exceeds the LDS budget go to the general kernel
    after the grouped ones (one identity with 200 rules, three with 20)."""
    from cilium_amd import api
    rng = np.random.default_rng(9)
    groups = []
    for g, k in enumerate((200, 20, 20, 20)):
        rules = [gen.cfg2_rules(int(x), 1)[0] for x in rng.integers(0, 4096, size=k)]
        groups.append(api.port_rule(remote_policies=[256 + g], http=api.http_rules_from_api(rules)))
    pol = api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(80, groups)]))
    reqs = gen.http_requests(80_000, 123)
    arena, offs, lens = gen.pack(reqs)
    conns = gen.make_conns(20, 0, 80, True, gen.PROTO_HTTP, np.array([256, 257, 258, 259] * 4 + [9000] * 4))
    cids = rng.integers(0, 20, size=len(reqs)).astype(np.uint32)
    w = gen.Workload("big-images", arena, offs, lens, cids, conns, pol, {})
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    st = engine.stats()
    assert st["http_image_bytes"] > 40_000, st  # the 200-rule image is over the 32 KiB budget
    got = engine.classify(w.arena, w.offsets, w.lengths, w.conn_ids)
    assert_same(got, oracle.classify_workload(w, 16), w)
