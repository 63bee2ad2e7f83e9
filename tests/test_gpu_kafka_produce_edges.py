"""Produce requests at the edges of kafka_classify_kernel's message-set walk
(the 36-byte window path, its exact fallback and the staged CRC batches)
against the oracle, bit-exact.

These streams put every case in front of both paths and every block / word
boundary of the CRC: messages of every length mod 64, keys long enough that
the value length lies past the message's first 64 bytes, empty sets and empty
messages, trailing bytes in a set, sets past the request's end, many sets per
request, bad CRCs at every position, codecs 1-3, and every arena alignment
(vendor/github.com/optiopay/kafka/proto/messages.go:363-494,1591-1647).
(Written in round 6 for a flat per-lane message loop, measured slower and not
kept; DESIGN.md §5 Kafka.)"""
import struct

import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, DENY, PROTO_KAFKA

from test_gpu_http import assert_same, both

pytestmark = pytest.mark.gpu


def _set_bytes(rng, v, mode):
    """One partition's message set and how it is broken (mode)."""
    msgs = []
    for _ in range(int(rng.integers(0, 7))):
        key = None
        r = rng.random()
        if r < 0.3:
            key = bytes(rng.integers(0, 256, size=int(rng.integers(0, 120)), dtype=np.uint8))
        elif r < 0.4:
            key = b""
        vl = int(rng.integers(0, 400)) if rng.random() < 0.8 else int(rng.integers(0, 16))
        val = None if rng.random() < 0.05 else bytes(rng.integers(0, 256, size=vl, dtype=np.uint8))
        attr = 0
        if mode == "codec":
            attr = int(rng.integers(0, 4))
        msgs.append(gen.k_message(val, key=key, version=v, attributes=attr,
                                  bad_crc=(mode == "crc" and rng.random() < 0.3)))
    ms = b"".join(msgs)
    if mode == "tail":  # trailing bytes after the last message
        ms += bytes(rng.integers(0, 256, size=int(rng.integers(1, 40)), dtype=np.uint8))
    if mode == "cut" and len(ms) > 8:  # the set's last message cut short
        ms = ms[: int(rng.integers(1, len(ms)))]
    return ms


def produce_edge(n, seed):
    rng = np.random.default_rng(seed)
    topics = gen.kafka_topics()
    modes = ["ok"] * 6 + ["crc", "tail", "cut", "codec", "bigset", "many"]
    out = []
    for i in range(n):
        v = int(rng.integers(0, 4))
        mode = modes[int(rng.integers(0, len(modes)))]
        nt = int(rng.integers(0, 4)) if mode != "many" else int(rng.integers(3, 7))
        body = b""
        if v >= 3:
            body += gen.k_str("tx" if rng.random() < 0.5 else None)
        body += struct.pack(">hi", -1, 1000) + struct.pack(">i", nt)
        for _ in range(nt):
            body += gen.k_str(topics[int(rng.integers(0, 1000))])
            npart = int(rng.integers(0, 3)) if mode != "many" else int(rng.integers(2, 4))
            body += struct.pack(">i", npart)
            for p in range(npart):
                ms = _set_bytes(rng, v, mode)
                size = len(ms)
                if mode == "bigset" and rng.random() < 0.5:
                    size += int(rng.integers(1, 5000))  # the set runs past the request
                body += struct.pack(">ii", p, size) + ms
        payload = struct.pack(">hhi", 0, v, i) + gen.k_str("client-%02d" % (i % 16)) + body
        req = struct.pack(">i", len(payload)) + payload
        out.append(req)
    # every arena alignment: a random 0-15 byte gap before each request
    pads = rng.integers(0, 16, size=n)
    reqs = [bytes(int(p)) + r for p, r in zip(pads, out)]
    arena, offs, lens = gen.pack(reqs)
    offs = offs + pads.astype(np.uint64)
    lens = lens - pads.astype(np.uint32)
    conn_ids = rng.integers(0, 256, size=n).astype(np.uint32)
    conns = gen.make_conns(256, 0, 9092, True, PROTO_KAFKA, 2000 + np.arange(256))
    return gen.Workload("produce-edge", arena, offs, lens, conn_ids, conns, gen.cfg3_policy())


@pytest.mark.parametrize("seed", [1, 2])
def test_produce_edges(engine, oracle, seed):
    w = produce_edge(12000, seed)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    v = got[0]
    assert (v == ALLOW).sum() > 100 and (v == DENY).sum() > 100


def test_produce_block_boundaries(engine, oracle):
    """One message per set, its value length swept so the message ends at every
    byte of a 64-byte block, at every arena alignment and both message formats."""
    topics = gen.kafka_topics()
    reqs = []
    for v in (0, 1):
        for vl in range(0, 200):
            for key in (None, b"k" * (vl % 70)):
                msgs = [gen.k_message(bytes([vl & 0xFF]) * vl, key=key, version=v),
                        gen.k_message(b"q" * ((vl * 7) % 90), version=v)]
                body = struct.pack(">hi", -1, 1000) + struct.pack(">i", 1) + gen.k_str(topics[vl % 500])
                body += struct.pack(">i", 1) + struct.pack(">ii", 0, len(b"".join(msgs))) + b"".join(msgs)
                payload = struct.pack(">hhi", 0, v, vl) + gen.k_str("client-01") + body
                reqs.append(struct.pack(">i", len(payload)) + payload)
    pads = [i % 16 for i in range(len(reqs))]
    arena, offs, lens = gen.pack([bytes(p) + r for p, r in zip(pads, reqs)])
    pads = np.array(pads)
    offs = offs + pads.astype(np.uint64)
    lens = lens - pads.astype(np.uint32)
    n = len(reqs)
    conns = gen.make_conns(1, 0, 9092, True, PROTO_KAFKA, [2000])
    w = gen.Workload("blocks", arena, offs, lens, np.zeros(n, np.uint32), conns, gen.cfg3_policy())
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    assert (got[0] == ALLOW).sum() > 0
