"""Compressed Kafka message sets in the oracle (no GPU).

readMessageSet (vendor/github.com/optiopay/kafka/proto/messages.go:460-489)
gunzips (Go 1.10 compress/gzip) or snappy-decodes (vendor/github.com/golang/
snappy, proto/snappy.go xerial framing) a message whose attributes & 3 is 1 or
2 and reads the result as a message set, recursively; any decode error fails
the request.  The reference holds no compressed vectors, so parity here is
pinned by construction: streams built with Python's gzip/zlib and a test
snappy encoder (cilium_amd/gen.py), decoded bytes compared with zlib's, and
the verdict of a compressed request compared with the same request
uncompressed.  Parity unpinned beyond that (no Go toolchain here).
"""
import gzip
import struct
import zlib

import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, PARSE_ERROR, PROTO_KAFKA

import refpy


def rng_data(rng, n, alphabet=None):
    if alphabet is None:
        return bytes(rng.integers(0, 256, n, dtype=np.uint8))
    return bytes(rng.choice(np.frombuffer(alphabet, np.uint8), n))


def gz_header(flags=0, extra=b"", name=b"", comment=b"", hcrc=False):
    h = bytes([0x1F, 0x8B, 8, flags | (0x02 if hcrc else 0)]) + b"\0\0\0\0\0\xff"
    if flags & 0x04:
        h += struct.pack("<H", len(extra)) + extra
    if flags & 0x08:
        h += name + b"\0"
    if flags & 0x10:
        h += comment + b"\0"
    if hcrc:
        h += struct.pack("<H", zlib.crc32(h) & 0xFFFF)
    return h


def gz_member(data, level=6, **hdr):
    c = zlib.compressobj(level, zlib.DEFLATED, -15)
    body = c.compress(data) + c.flush()
    return gz_header(**hdr) + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)


@pytest.mark.parametrize("level", [0, 1, 6, 9])
def test_gunzip_round_trip(level):
    rng = np.random.default_rng(level)
    for n in (0, 1, 100, 5000, 70000):
        for alpha in (None, b"ab", b"abcdefghij klmnop"):
            d = rng_data(rng, n, alpha)
            assert refpy.gunzip(gzip.compress(d, compresslevel=level)) == d
            assert refpy.gunzip(gz_member(d, level)) == d


def test_gunzip_header_fields_and_members():
    d = b"kafka message set bytes " * 50
    for hdr in (dict(flags=0x04, extra=b"xyz"), dict(flags=0x08, name=b"file.bin"), dict(flags=0x10, comment=b"c"),
                dict(flags=0x1C, extra=b"\1\2", name=b"n", comment=b"cc", hcrc=True), dict(hcrc=True)):
        assert refpy.gunzip(gz_member(d, **hdr)) == d
    # readString: 511 name bytes + NUL fit Go's 512-byte buffer, 512 do not
    assert refpy.gunzip(gz_member(d, flags=0x08, name=b"a" * 511)) == d
    assert refpy.gunzip(gz_member(d, flags=0x08, name=b"a" * 512)) is None
    # a wrong header CRC
    m = bytearray(gz_member(d, hcrc=True))
    m[10] ^= 1
    assert refpy.gunzip(bytes(m)) is None
    # multistream: members concatenate; an empty member is fine
    assert refpy.gunzip(gz_member(d) + gz_member(b"") + gz_member(b"tail")) == d + b"tail"


def test_gunzip_member_history_is_reset():
    """Each member gets a fresh flate reader (gunzip.go readHeader:
    Reset(z.r, nil)): a back-reference into the previous member's output is
    corrupt input, even though the bytes are there."""
    d = b"0123456789abcdef" * 200
    second = gen._gz_member(d[1600:], zdict=d[:1600])
    assert refpy.gunzip(gen._gz_member(d[:1600]) + second) is None
    assert refpy.gunzip(gen._gz_member(d[:1600]) + gen._gz_member(d[1600:])) == d


def test_gunzip_errors():
    d = bytes(range(256)) * 40
    m = gz_member(d)
    assert refpy.gunzip(b"") is None                 # io.EOF from NewReader
    for cut in (1, 5, 9, 10, 11, len(m) // 2, len(m) - 8, len(m) - 1):
        assert refpy.gunzip(m[:cut]) is None, cut    # every proper prefix
    for k in range(1, 10):
        assert refpy.gunzip(m + b"\0" * k) is None   # a partial next header
    assert refpy.gunzip(m + b"\0" * 10) is None      # not a gzip header
    bad = bytearray(m)
    bad[-8] ^= 1                                     # CRC32
    assert refpy.gunzip(bytes(bad)) is None
    bad = bytearray(m)
    bad[-4] ^= 1                                     # ISIZE
    assert refpy.gunzip(bytes(bad)) is None
    bad = bytearray(m)
    bad[2] = 7                                       # CM
    assert refpy.gunzip(bytes(bad)) is None
    assert refpy.gunzip(m, cap=len(d) - 1) is None   # larger than readMessageSet accepts
    assert refpy.gunzip(m, cap=len(d)) == d


def test_inflate_bit_flips_agree_with_zlib():
    """Corrupted DEFLATE bodies: Go's inflate and zlib reject the same streams
    (a single-code code-length code, where they differ, always fails later in
    Go too), and decode the survivors to the same bytes."""
    rng = np.random.default_rng(7)
    agree = 0
    for trial in range(600):
        d = rng_data(rng, int(rng.integers(1, 3000)), b"abcab cabbage\n" if trial % 2 else None)
        c = zlib.compressobj(int(rng.integers(1, 10)), zlib.DEFLATED, -15)
        body = bytearray(c.compress(d) + c.flush())
        for _ in range(int(rng.integers(1, 4))):
            i = int(rng.integers(0, len(body)))
            body[i] ^= 1 << int(rng.integers(0, 8))
        try:
            z = zlib.decompressobj(-15)
            out = z.decompress(bytes(body))
            zok = z.eof and not z.unused_data
        except zlib.error:
            zok, out = False, None
        # wrap with a trailer that matches zlib's output, so only the body decides
        trailer = struct.pack("<II", zlib.crc32(out or b"") & 0xFFFFFFFF, len(out or b"") & 0xFFFFFFFF)
        got = refpy.gunzip(gz_header() + bytes(body) + trailer)
        if zok:
            assert got == out, trial
        else:
            # zlib stopped early (error, or a stream ending before the data):
            # the restatement must not produce zlib's bytes as a full member
            assert got is None or not z.eof, trial
        agree += 1
    assert agree == 600


def test_snappy_round_trip_and_xerial():
    rng = np.random.default_rng(3)
    for n in (0, 1, 59, 60, 61, 255, 256, 257, 4000, 70000):
        for alpha in (None, b"xy", b"the quick brown fox "):
            d = rng_data(rng, n, alpha)
            assert refpy.unsnappy(gen.snappy_block(d)) == d
            assert refpy.unsnappy(gen.snappy_block(d, copies=False)) == d
            assert refpy.unsnappy(gen.snappy_xerial(d, chunk=1000)) == d


def test_snappy_errors():
    d = b"abcdabcdabcdabcd" * 10
    b = gen.snappy_block(d)
    assert refpy.unsnappy(b"") is None                        # no varint
    assert refpy.unsnappy(b"\x80") is None                    # unterminated varint
    assert refpy.unsnappy(b"\xff" * 10 + b"\x01") is None     # varint overflow
    assert refpy.unsnappy(b"\x80\x80\x80\x80\x10") is None    # > 0xffffffff
    assert refpy.unsnappy(b"\x00") == b""                     # empty block
    for cut in range(1, len(b)):
        assert refpy.unsnappy(b[:cut]) is None, cut           # short output or a cut tag
    assert refpy.unsnappy(b"\x05" + bytes([(3 << 2)]) + b"abcd") is None  # d != len(dst)
    assert refpy.unsnappy(b"\x04\x01\x00") is None            # copy with offset 0... and d < offset
    assert refpy.unsnappy(b"\x08" + bytes([(3 << 2)]) + b"abcd" + bytes([1, 8])) is None  # offset 8 > d
    assert refpy.unsnappy(b"\x08" + bytes([(3 << 2)]) + b"abcd" + bytes([1, 4])) == b"abcdabcd"
    # xerial: version must be 1; 12..15 bytes decode to nothing; cut chunks fail
    x = gen.snappy_xerial(d)
    assert refpy.unsnappy(x[:8] + struct.pack(">i", 2) + x[12:]) is None
    assert refpy.unsnappy(x[:11]) is None
    assert refpy.unsnappy(x[:12]) == b"" and refpy.unsnappy(x[:15]) == b""
    assert refpy.unsnappy(x[:18]) is None
    assert refpy.unsnappy(x[:-1]) is None
    assert refpy.unsnappy(b, cap=len(d) - 1) is None


# ---------------------------------------------------------------- verdicts
TOPIC = "orders"


def policy():
    rules = [api.PortRuleKafka(api_key="produce", topic=TOPIC)]
    return api.policy_set(api.network_policy("ep", 1, ingress=[(9092, [api.port_rule(kafka=rules)])]))


def verdicts(reqs):
    conns = gen.make_conns(1, 0, 9092, True, PROTO_KAFKA, [7], 9)
    arena, offs, lens = gen.pack(reqs)
    v, r, c = refpy.Policy(policy()).classify(conns, arena, offs, lens, np.zeros(len(reqs), np.uint32))
    return list(v)


def inner_set(rng, version, k=3):
    return b"".join(gen.k_message(rng_data(rng, int(rng.integers(0, 300)), b"payload "), version=version)
                    for _ in range(k))


@pytest.mark.parametrize("version", [0, 1, 2])
def test_compressed_produce_same_verdict_as_plain(version):
    rng = np.random.default_rng(100 + version)
    reqs, want = [], []
    for topic in (TOPIC, "other"):
        for codec, xerial in ((1, False), (2, False), (2, True)):
            inner = inner_set(rng, version)
            msg = gen.k_compressed(inner, codec, version=version, xerial=xerial)
            reqs.append(gen.k_produce(version, 1, "c", [(topic, [(0, [msg])])]))
            plain = gen.k_produce(version, 1, "c", [(topic, [(0, [inner])])])
            want.append(verdicts([plain])[0])
    assert verdicts(reqs) == want
    assert set(want) == {ALLOW, DENY}


def test_compressed_corrupt_is_parse_error():
    rng = np.random.default_rng(5)
    inner = inner_set(rng, 0)
    good = gzip.compress(inner)
    cases = [good[:-1], good[:20], b"", b"\x1f\x8b\x08", good + b"\0\0\0",
             gen.snappy_block(inner)[:-2], gen.snappy_xerial(inner)[:10], b"\x82SNAPPY\x00\0\0\0\2\0\0\0\1"]
    reqs = []
    for i, value in enumerate(cases):
        codec = 1 if i < 5 else 2
        msg = gen.k_message(value, attributes=codec)
        reqs.append(gen.k_produce(0, 1, "c", [(TOPIC, [(0, [msg])])]))
    assert verdicts(reqs) == [PARSE_ERROR] * len(cases)


def test_compressed_nested_and_inner_quirks():
    rng = np.random.default_rng(9)
    inner = inner_set(rng, 0)
    lvl1 = gen.k_compressed(inner, 2)
    lvl2 = gen.k_compressed(lvl1, 1)
    lvl3 = gen.k_compressed(lvl2 + gen.k_message(b"plain"), 2, xerial=True)
    ok = gen.k_produce(0, 1, "c", [(TOPIC, [(0, [lvl3])])])
    # inner set with a bad CRC: readMessageSet stops there without an error
    crc_stop = gen.k_compressed(gen.k_message(b"x", bad_crc=True) + gen.k_message(b"y"), 1)
    # a corrupt stream nested two levels down fails the request
    deep_bad = gen.k_compressed(gen.k_message(b"\x1f\x8b\x08\0garbage", attributes=1), 2)
    # more than 6,553,500 decoded bytes (messages.go:369-371)
    big = gen.k_message(gzip.compress(b"\0" * 6_553_501), attributes=1)
    fits = gen.k_message(gzip.compress(gen.k_message(b"\0" * 6_553_400)), attributes=1)
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [m])])]) for m in (crc_stop, deep_bad, big, fits)]
    assert verdicts([ok] + reqs) == [ALLOW, ALLOW, PARSE_ERROR, PARSE_ERROR, ALLOW]


def test_compressed_then_more_messages():
    """The outer set goes on after a compressed message: a later plain message
    with a short value field is still an error, a later bad CRC a silent stop."""
    rng = np.random.default_rng(11)
    comp = gen.k_compressed(inner_set(rng, 0), 1)
    later_ok = gen.k_message(b"after")
    later_stop = gen.k_message(b"after", bad_crc=True)
    reqs = [gen.k_produce(0, 1, "c", [(TOPIC, [(0, [comp, later_ok])])]),
            gen.k_produce(0, 1, "c", [(TOPIC, [(0, [comp, later_stop, comp])])])]
    assert verdicts(reqs) == [ALLOW, ALLOW]
