"""Compressed Kafka message sets on the GPU: kafka_classify_kernel lists the
requests, kafka_inflate_kernel gunzips / snappy-decodes and reads the inner
sets (messages.go:460-489); verdicts bit-exact against the oracle.

The reference holds no compressed vectors: parity unpinned beyond the oracle
restatement, which tests/test_kafka_compressed_host.py pins against zlib and
against the same requests sent uncompressed.
"""
import gzip
import struct
import zlib

import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, PARSE_ERROR, PROTO_KAFKA

from test_gpu_http import assert_same, both, wl_from_reqs
from test_kafka_compressed_host import inner_set, policy, rng_data, TOPIC

pytestmark = pytest.mark.gpu


def conns():
    return gen.make_conns(1, 0, 9092, True, PROTO_KAFKA, [7], 9)


def run(engine, oracle, reqs):
    w = wl_from_reqs(reqs, policy(), conns())
    got, ref = both(engine, oracle, w, 1)
    assert_same(got, ref, w)
    return got[0].tolist()


def test_same_verdict_as_plain(engine, oracle):
    rng = np.random.default_rng(1)
    reqs, plain = [], []
    for version in (0, 1, 2):
        for topic in (TOPIC, "other"):
            for codec, xerial in ((1, False), (2, False), (2, True)):
                inner = inner_set(rng, version)
                reqs.append(gen.k_produce(version, 1, "c", [(topic, [(0, [gen.k_compressed(inner, codec, version=version,
                                                                                           xerial=xerial)])])]))
                plain.append(gen.k_produce(version, 1, "c", [(topic, [(0, [inner])])]))
    assert run(engine, oracle, reqs) == run(engine, oracle, plain)


def test_corrupt_and_nested(engine, oracle):
    rng = np.random.default_rng(5)
    inner = inner_set(rng, 0)
    good = gzip.compress(inner)
    corrupt = [good[:-1], good[:20], b"", b"\x1f\x8b\x08", good + b"\0\0\0",
               gen.snappy_block(inner)[:-2], gen.snappy_xerial(inner)[:10], b"\x82SNAPPY\x00\0\0\0\2\0\0\0\1"]
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [gen.k_message(v, attributes=1 if i < 5 else 2)])])])
            for i, v in enumerate(corrupt)]
    lvl3 = gen.k_compressed(gen.k_compressed(gen.k_compressed(inner, 2), 1) + gen.k_message(b"plain"), 2, xerial=True)
    crc_stop = gen.k_compressed(gen.k_message(b"x", bad_crc=True) + gen.k_message(b"y"), 1)
    deep_bad = gen.k_compressed(gen.k_message(b"\x1f\x8b\x08\0garbage", attributes=1), 2)
    comp = gen.k_compressed(inner, 1)
    for m in ([lvl3], [crc_stop], [deep_bad], [comp, gen.k_message(b"after")],
              [comp, gen.k_message(b"after", bad_crc=True), comp]):
        reqs.append(gen.k_produce(0, 1, "c", [(TOPIC, [(0, m)])]))
    got = run(engine, oracle, reqs)
    assert got[:len(corrupt)] == [PARSE_ERROR] * len(corrupt)
    assert got[len(corrupt):] == [ALLOW, ALLOW, PARSE_ERROR, ALLOW, ALLOW]


def test_size_limit(engine, oracle):
    """More than 6,553,500 decoded bytes fail (messages.go:369-371); just
    under it decodes, also one level down inside a snappy set."""
    big = gen.k_message(gzip.compress(b"\0" * 6_553_501), attributes=1)
    fits = gen.k_message(gzip.compress(gen.k_message(b"\0" * 6_553_400)), attributes=1)
    snap_big = gen.k_message(gen.snappy_block(b"\1" * 6_553_501, copies=False), attributes=2)
    nested = gen.k_compressed(gen.k_message(gzip.compress(gen.k_message(b"\0" * 3_000_000)), attributes=1), 2)
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [m])])]) for m in (big, fits, snap_big, nested)]
    assert run(engine, oracle, reqs) == [PARSE_ERROR, ALLOW, PARSE_ERROR, ALLOW]


def test_gzip_shapes(engine, oracle):
    """Stored / fixed / dynamic blocks, header fields, members, and a member
    whose back-reference reaches into the previous member (Go resets the
    flate reader per member: corrupt)."""
    rng = np.random.default_rng(8)
    inner = b"".join(gen.k_message(rng_data(rng, 2000, b"abcd efgh"), version=1) for _ in range(5))
    vals = [gen._gz_member(inner, level=lv, strategy=st)
            for lv in (0, 1, 6, 9) for st in (0, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE)]
    vals += [gen._gz_member(inner, flags=0x1C, extra=b"e" * 300, name=b"n" * 511, comment=b"c", hcrc=True),
             gen._gz_member(inner, flags=0x08, name=b"n" * 512),
             gen._gz_member(inner) + gen._gz_member(b"") + gen._gz_member(inner[:5000]),
             gen._gz_member(inner[:3000]) + gen._gz_member(inner[3000:], zdict=inner[:3000])]
    reqs = [gen.k_produce(1, 1, "c", [(TOPIC, [(0, [gen.k_message(v, version=1, attributes=1)])])]) for v in vals]
    got = run(engine, oracle, reqs)
    assert got[:16] == [ALLOW] * 16
    assert got[16:] == [ALLOW, PARSE_ERROR, ALLOW, PARSE_ERROR]


def test_snappy_long_offsets(engine, oracle):
    """A copy-4 tag reaching further back than the 64 KiB LDS history ring."""
    rng = np.random.default_rng(9)
    msg = gen.k_message(rng_data(rng, 300))
    body = msg + gen.k_message(bytes(70000))  # 64 bytes copied from 100000 back = start of `msg`
    blk = gen.snappy_far_copy(body, 100000)
    dec_len = 100000 + 64
    # the decoded set: msg, the zero message, zero padding (offset 0, size 0:
    # the set ends), then the copy -- only decodability matters for the verdict
    ok = gen.k_message(blk, attributes=2)
    bad = gen.k_message(blk[:-1] + bytes([blk[-1] ^ 0x7F]), attributes=2)  # offset > decoded length
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [m])])]) for m in (ok, bad)]
    assert dec_len > 65536
    assert run(engine, oracle, reqs) == [ALLOW, PARSE_ERROR]


def test_bit_flips(engine, oracle):
    """Single bit flips in gzip and snappy values (message CRC recomputed), so
    every decoder error path is reached; device and oracle agree on each."""
    rng = np.random.default_rng(10)
    inner = inner_set(rng, 0, k=4)
    reqs = []
    for codec, value in ((1, gzip.compress(inner, 6)), (1, gen._gz_member(inner, 1, zlib.Z_FIXED)),
                         (2, gen.snappy_block(inner)), (2, gen.snappy_xerial(inner, 300))):
        for _ in range(150):
            v = bytearray(value)
            i = int(rng.integers(0, len(v)))
            v[i] ^= 1 << int(rng.integers(0, 8))
            reqs.append(gen.k_produce(0, 1, "c", [(TOPIC, [(0, [gen.k_message(bytes(v), attributes=codec)])])]))
    got = run(engine, oracle, reqs)
    assert got.count(PARSE_ERROR) > 100 and got.count(ALLOW) > 10


@pytest.mark.parametrize("seed", [0, 1])
def test_random_compressed_stream(engine, oracle, seed):
    reqs = gen.kafka_compressed_requests(3000, 4242 + seed)
    w = wl_from_reqs(reqs, gen.cfg3_policy(), gen.make_conns(64, 0, 9092, True, PROTO_KAFKA, 2000 + np.arange(64)),
                     np.random.default_rng(seed).integers(0, 64, len(reqs)))
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    v = got[0]
    assert (v == PARSE_ERROR).sum() > 100 and ((v == ALLOW) | (v == DENY)).sum() > 1000


def test_mixed_with_plain_cfg3(engine, oracle):
    """Compressed requests inside a cfg3 stream: the plain requests' verdicts
    are untouched, the compressed ones decided."""
    w3 = gen.kafka_workload(4000)
    reqs = [bytes(w3.arena[int(o):int(o) + int(L)]) for o, L in zip(w3.offsets, w3.lengths)]
    z = gen.kafka_compressed_requests(500, 99)
    mixed = []
    for i, r in enumerate(reqs):
        mixed.append(r)
        if i % 8 == 0:
            mixed.append(z[i // 8])
    w = wl_from_reqs(mixed, gen.cfg3_policy(), w3.conns,
                     np.random.default_rng(3).integers(0, len(w3.conns), len(mixed)))
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)


def test_snappy_decode_go_vectors(engine, oracle):
    """The snappy vectors derived from the reference's vendored decoder
    (tests/test_snappy_decode_go.py) as snappy-coded messages of produce
    requests: the inflate kernel's verdicts equal the oracle's, and a vector
    Decode rejects makes its request PARSE_ERROR."""
    from test_snappy_decode_go import VECTORS
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [gen.k_message(src, attributes=2)])])]) for _, src, _, _ in VECTORS]
    got = run(engine, oracle, reqs)
    for (name, _, expected, where), v in zip(VECTORS, got):
        if expected is None:
            assert v == PARSE_ERROR, f"{name}: {where}"
