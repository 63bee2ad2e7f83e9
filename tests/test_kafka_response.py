"""Kafka deny responses (host code in the product library; no GPU needed).

pkg/proxy/kafka.go:249-261 answers a denied request with
req.CreateResponse(proto.ErrTopicAuthorizationFailed) (pkg/kafka/request.go:
158-182, response.go:81-315), encoded by the vendored optiopay *Resp.Bytes
(vendor/github.com/optiopay/kafka/proto/messages.go:610, 911, 1117, 1342, 1531,
1716, 1975).  The expected bytes below are an independent Python restatement
of those encoders; the reference's own test pins the produce case
(pkg/proxy/kafka_test.go:184-258: errno 29 for the disallowed topic).
Parity beyond that case is unpinned (no reference test encodes the others)."""
import struct

import numpy as np
import pytest

from cilium_amd import _lib, gen

ERR = 29
ZERO_TIME_MS = -6795364578871  # time.Time{}.UnixNano()/1e6 with Go's int64 wrap


def s(x):
    b = x.encode() if isinstance(x, str) else x
    return struct.pack(">h", len(b)) + b


def frame(corr, body):
    return struct.pack(">ii", 4 + len(body), corr) + body


def expect(kind, v, corr, topics=None, meta=None):
    """topics: [(name, [pids])]; meta: list of names or None (null)."""
    b = b""
    if kind == 0:
        b += struct.pack(">i", len(topics))
        for n, ps in topics:
            b += s(n) + struct.pack(">i", len(ps))
            for p in ps:
                b += struct.pack(">ihq", p, ERR, 0) + (struct.pack(">q", 0) if v >= 2 else b"")
        if v >= 1:
            b += struct.pack(">i", 0)
    elif kind == 1:
        b += struct.pack(">i", 0) if v >= 1 else b""
        b += struct.pack(">i", len(topics))
        for n, ps in topics:
            b += s(n) + struct.pack(">i", len(ps))
            for p in ps:
                b += struct.pack(">ihq", p, ERR, 0)
                if v >= 4:
                    b += struct.pack(">q", 0) + (struct.pack(">q", 0) if v >= 5 else b"") + struct.pack(">i", -1)
                b += struct.pack(">i", 0)
    elif kind == 2:
        b += struct.pack(">i", 0) if v >= 2 else b""
        b += struct.pack(">i", len(topics))
        for n, ps in topics:
            b += s(n) + struct.pack(">i", len(ps))
            for p in ps:
                b += struct.pack(">ih", p, ERR) + (struct.pack(">q", ZERO_TIME_MS) if v >= 1 else b"") + \
                    struct.pack(">i", 0)
    elif kind == 3:
        b += struct.pack(">i", 0) if v >= 3 else b""
        b += struct.pack(">i", 0) + (s("") if v >= 2 else b"") + (struct.pack(">i", 0) if v >= 1 else b"")
        if meta is None:
            b += struct.pack(">i", -1)
        else:
            b += struct.pack(">i", len(meta))
            for n in meta:
                b += struct.pack(">h", ERR) + s(n) + (b"\x00" if v >= 1 else b"") + struct.pack(">i", 0)
    elif kind == 8:
        b += struct.pack(">i", 0) if v >= 3 else b""
        b += struct.pack(">i", len(topics))
        for n, ps in topics:
            b += s(n) + struct.pack(">i", len(ps)) + b"".join(struct.pack(">ih", p, ERR) for p in ps)
    elif kind == 9:
        b += struct.pack(">i", 0) if v >= 3 else b""
        if topics is None:
            b += struct.pack(">i", -1)
        else:
            b += struct.pack(">i", len(topics))
            for n, ps in topics:
                b += s(n) + struct.pack(">i", len(ps))
                for p in ps:
                    b += struct.pack(">iq", p, 0) + s("") + struct.pack(">h", ERR)
        b += struct.pack(">h", 0) if v >= 2 else b""
    elif kind == 10:
        b += (struct.pack(">i", 0) if v >= 1 else b"") + struct.pack(">h", ERR) + (s("") if v >= 1 else b"") + \
            struct.pack(">i", 0) + s("") + struct.pack(">i", 0)
    return frame(corr, b)


TOPICS = [("alpha", [0, 3]), ("", [7]), ("gamma", [])]


@pytest.mark.parametrize("v", range(4))
def test_produce(v):
    t = [(n, [(p, [gen.k_message(b"x" * 10, version=v)]) for p in ps]) for n, ps in TOPICS]
    req = gen.k_produce(v, 11, "c", t, txn="t" if v >= 3 else None)
    assert _lib.kafka_deny_response(req) == expect(0, v, 11, TOPICS)


def test_produce_bad_crc_stops_the_set():
    """A CRC mismatch stops readMessageSet without draining it: the next
    partition id is read from inside the set (messages.go:431-435)."""
    msgs = [gen.k_message(b"a" * 20, bad_crc=True), gen.k_message(b"b" * 20)]
    req = gen.k_produce(0, 5, "c", [("t", [(1, msgs)])])
    # the decoder resumes right after the bad message and reads the topic's
    # remaining partition count from there; the result is whatever the
    # sequential decode gives -- here the request still decodes or not, and
    # the response (if any) must be self-consistent
    out = _lib.kafka_deny_response(req)
    assert out is None or struct.unpack(">i", out[:4])[0] == len(out) - 4


@pytest.mark.parametrize("v", range(6))
def test_fetch(v):
    req = gen.k_fetch(v, 12, "c", TOPICS)
    assert _lib.kafka_deny_response(req) == expect(1, v, 12, TOPICS)


@pytest.mark.parametrize("v", range(3))
def test_offsets(v):
    req = gen.k_offset(v, 13, "c", TOPICS)
    assert _lib.kafka_deny_response(req) == expect(2, v, 13, TOPICS)


@pytest.mark.parametrize("v", range(6))
@pytest.mark.parametrize("names", [None, [], ["a", "", "a"]])
def test_metadata(v, names):
    req = gen.k_metadata(v, 14, "c", names)
    assert _lib.kafka_deny_response(req) == expect(3, v, 14, meta=names)


@pytest.mark.parametrize("v", range(4))
def test_offset_commit(v):
    req = gen.k_offset_commit(v, 15, "c", "g", TOPICS)
    assert _lib.kafka_deny_response(req) == expect(8, v, 15, TOPICS)


@pytest.mark.parametrize("v", range(4))
@pytest.mark.parametrize("null", [False, True])
def test_offset_fetch(v, null):
    req = gen.k_offset_fetch(v, 16, "c", "g", None if null else TOPICS)
    assert _lib.kafka_deny_response(req) == expect(9, v, 16, None if null else TOPICS)


@pytest.mark.parametrize("v", range(2))
def test_consumer_metadata(v):
    req = gen.k_consumer_metadata(v, 17, "c", "g")
    assert _lib.kafka_deny_response(req) == expect(10, v, 17)


def test_untyped_and_broken_requests_get_no_response():
    assert _lib.kafka_deny_response(gen.k_request(18, 0, 1, "c", b"")) is None  # ApiVersions: request == nil
    assert _lib.kafka_deny_response(gen.k_fetch(0, 1, "c", TOPICS)[:20]) is None
    assert _lib.kafka_deny_response(b"\x00\x00\x00\x02\x00\x00") is None


def test_reference_disallowed_topic_case():
    """pkg/proxy/kafka_test.go:242-258 (produce v0, disallowedTopic, partition 0)."""
    msgs = [gen.k_message(b"first"), gen.k_message(b"second")]
    out = _lib.kafka_deny_response(gen.k_produce(0, 42, "tester", [("disallowedTopic", [(0, msgs)])]))
    size, corr, nt = struct.unpack(">iii", out[:12])
    assert (size, corr, nt) == (len(out) - 4, 42, 1)
    assert out[12:14 + 15] == s("disallowedTopic")
    assert struct.unpack(">iihq", out[29:47]) == (1, 0, 29, 0)


def test_correlation_cache_round_trip():
    """correlation_cache.go: forwarded requests get ids 1, 2, ...; responses
    carrying them get the client's original ids back; unknown ones pass."""
    cc = _lib.KafkaCorrelationCache()
    reqs = [gen.k_fetch(0, 1000 + i, "c", TOPICS) for i in range(5)]
    arena, offs, lens = gen.pack(reqs)
    arena = np.array(arena, np.uint8)
    ids = cc.requests(arena, offs, lens)
    assert ids.tolist() == [1, 2, 3, 4, 5] and len(cc) == 5
    for i, o in enumerate(offs):
        assert struct.unpack(">i", bytes(arena[o + 8:o + 12]))[0] == i + 1
        assert bytes(arena[o + 12:o + lens[i]]) == reqs[i][12:]  # nothing else touched
    # the broker answers 3, 1 and an id the proxy never issued
    resp = [expect(1, 0, 3, TOPICS), expect(1, 0, 1, TOPICS), expect(1, 0, 99, TOPICS)]
    rarena, roffs, rlens = gen.pack(resp)
    rarena = np.array(rarena, np.uint8)
    found = cc.responses(rarena, roffs, rlens)
    assert found.tolist() == [True, True, False]
    got = [struct.unpack(">i", bytes(rarena[o + 4:o + 8]))[0] for o in roffs]
    assert got == [1002, 1000, 99]
    assert len(cc) == 3
    assert cc.responses(rarena, roffs[:1], rlens[:1]).tolist() == [False]  # 3 is forgotten now
    assert cc.gc(10 ** 9) == 0 and cc.gc(0) == 3 and len(cc) == 0
    more = cc.requests(arena, offs[:2], lens[:2])
    assert more.tolist() == [6, 7]  # the sequence continues
