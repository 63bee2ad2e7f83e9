"""Kafka parity on the GPU: product vs oracle, bit-exact."""
import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, PROTO_KAFKA

from test_gpu_http import assert_same, both

pytestmark = pytest.mark.gpu


def test_kafka_kats(engine, oracle, kats):
    K = kats["kafka"]
    for case in K["cases"]:
        req = bytes.fromhex(K["requests"][case["request"]])
        pol = api.policy_set(api.network_policy("ep", 1, ingress=[(9092, [api.port_rule(kafka=case["rules"])])]))
        conns = gen.make_conns(1, 0, 9092, True, PROTO_KAFKA, [case.get("src_id", 7)])
        w = gen.Workload("kat", np.frombuffer(req, np.uint8).copy(), np.array([0], np.uint64),
                         np.array([len(req)], np.uint32), np.zeros(1, np.uint32), conns, pol)
        got, ref = both(engine, oracle, w, 1)
        assert got[0][0] == (ALLOW if case["expect"] == "ALLOW" else DENY), case
        assert_same(got, ref, w)


def test_cfg3_parity(engine, oracle):
    w = gen.kafka_workload(20000)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    v = got[0]
    assert (v == ALLOW).mean() > 0.1 and (v == DENY).mean() > 0.02


def test_kafka_adversarial_parity(engine, oracle):
    w = gen.kafka_workload(20000, seed=31337, adversarial=True)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    assert len(set(got[0].tolist())) >= 4


def test_mixed_http_kafka_batch(engine, oracle):
    """One batch, HTTP and Kafka connections interleaved; both kernels run."""
    h = gen.http_workload(2, 3000)
    k = gen.kafka_workload(3000)
    pol = {"policies": [h.policy["policies"][0], dict(k.policy["policies"][0], name="10.0.0.2")]}
    conns = np.concatenate([h.conns, k.conns])
    conns["policy"][len(h.conns):] = 1
    arena = np.concatenate([h.arena, k.arena])
    offs = np.concatenate([h.offsets, k.offsets + np.uint64(len(h.arena))])
    lens = np.concatenate([h.lengths, k.lengths])
    cids = np.concatenate([h.conn_ids, k.conn_ids + np.uint32(len(h.conns))])
    perm = np.random.default_rng(1).permutation(len(offs))
    w = gen.Workload("mixed", arena, offs[perm], lens[perm], cids[perm], conns, pol)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)


def test_kafka_all_kinds_parity(engine, oracle):
    """Every decoder the reference has (Produce, Fetch, ListOffsets, Metadata,
    OffsetCommit, OffsetFetch, ConsumerMetadata) at every version its fields
    depend on, empty / null topic arrays, empty topic names, truncated and
    size-edited frames, untyped kinds."""
    w = gen.kafka_workload(30000, seed=99, all_kinds=True)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    assert len(set(got[0].tolist())) >= 4
