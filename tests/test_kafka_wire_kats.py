"""Hand-derived wire KATs for Kafka decoder quirks (no reference vector holds
these: derived line by line from the vendored decoder, so "parity unpinned"
in the sense of DESIGN.md §2 -- the expectations are the derivation, checked
against the oracle here and against the device in the GPU variant).

  ReadProduceReq  vendor/github.com/optiopay/kafka/proto/messages.go:1591-1647
  readMessageSet  messages.go:363-494
  decoder         serialization.go (sticky err, io.ReadFull semantics)

The produce decoder reads partition id / set size through its own decoder
and hands the *same reader* to readMessageSet, which wraps it in a
LimitReader and a fresh decoder: a short read or a bad CRC inside the set
ends the set without an error, and the outer decoder continues from wherever
the set stopped.
"""
import struct

import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, PARSE_ERROR, PROTO_KAFKA

import refpy

T1 = "orders"


def policy(topic_rule=True):
    rules = [api.PortRuleKafka(role="produce", topic=T1)] if topic_rule else [api.PortRuleKafka(api_key="produce")]
    return api.policy_set(api.network_policy("ep", 1, ingress=[(9092, [api.port_rule(kafka=rules)])]))


def produce_raw(body_after_acks):
    """Produce v0 request: header, client "c", acks/timeout, then the given bytes."""
    return gen.k_request(0, 0, 1, "c", struct.pack(">hi", -1, 1000) + body_after_acks)


def topic_hdr(name, nparts):
    return gen.k_str(name) + struct.pack(">i", nparts)


def part_hdr(pid, set_size):
    return struct.pack(">ii", pid, set_size)


def cases():
    m1 = gen.k_message(b"x" * 40)
    m2 = gen.k_message(b"y" * 40)
    bad = gen.k_message(b"z" * 40, bad_crc=True)
    out = []
    # A. one partition whose set is cut short by the end of the request: the
    # message's io.ReadFull fails with ErrUnexpectedEOF -> readMessageSet
    # returns (set, nil) (:414-419); no partitions follow, dec.Err() is nil
    # (:1643) -> parsed, topics [orders] -> ALLOW under the topic rule.
    body = struct.pack(">i", 1) + topic_hdr(T1, 1) + part_hdr(0, len(m1) + len(m2)) + m1 + m2[:20]
    out.append(("short set, last partition", produce_raw(body), True, ALLOW))
    # B. the same cut inside the first of two partitions: the second partition's
    # ID read hits EOF (:1631-1633) -> error -> PARSE_ERROR.
    body = struct.pack(">i", 1) + topic_hdr(T1, 2) + part_hdr(0, len(m1) + len(m2)) + m1 + m2[:20]
    out.append(("short set, then a partition", produce_raw(body), True, PARSE_ERROR))
    # C. a bad CRC ends the set without draining it (:427-431); the outer
    # decoder then reads topic 2 from the unread message's bytes: its offset
    # field (8 zero bytes) decodes as name "" (int16 0) and a partition count
    # of 0 (int32 0) -> parsed, topics [orders, ""] -> the topic rule does not
    # cover "" -> DENY; a topic-less produce rule -> ALLOW.
    body = struct.pack(">i", 2) + topic_hdr(T1, 1) + part_hdr(0, len(bad) + len(m2)) + bad + m2
    out.append(("bad crc, next topic from the set", produce_raw(body), True, DENY))
    out.append(("bad crc, topic-less rule", produce_raw(body), False, ALLOW))
    # D. a message of size 4 (just the CRC) is appended and ends the set
    # (:421-425); the rest of the set is read as the next partition: 8 zero
    # bytes = partition id 0, set size 0 -> an empty set -> parsed -> ALLOW.
    tiny = struct.pack(">qi", 0, 4) + b"\0\0\0\0"
    body = (struct.pack(">i", 1) + topic_hdr(T1, 2) + part_hdr(0, len(tiny) + 8) + tiny + bytes(8))
    out.append(("4-byte message then a partition", produce_raw(body), True, ALLOW))
    # E. a null set (size -1) reads nothing (:365-367); the next partition
    # follows directly -> parsed -> ALLOW.
    body = struct.pack(">i", 1) + topic_hdr(T1, 2) + part_hdr(0, -1) + part_hdr(1, len(m1)) + m1
    out.append(("null set", produce_raw(body), True, ALLOW))
    # F. a set size over 6,553,500 is a messageSizeError (:369-371) -> PARSE_ERROR,
    # even with the bytes absent.
    body = struct.pack(">i", 1) + topic_hdr(T1, 1) + part_hdr(0, 6_553_501)
    out.append(("oversized set", produce_raw(body), True, PARSE_ERROR))
    # G. a message size field <= 0 ends the set (:405-408); the outer decoder
    # continues after the 12 bytes read: the next 6 bytes of the set are read
    # as topic 2 = name "" + 0 partitions -> topics [orders, ""] -> DENY.
    zero = struct.pack(">qi", 0, 0) + bytes(6)
    body = struct.pack(">i", 2) + topic_hdr(T1, 1) + part_hdr(0, len(zero)) + zero
    out.append(("zero message size", produce_raw(body), True, DENY))
    # H. a valid message followed by a key-length field that runs past the
    # message (msgdec short read inside the message) -> msgdec.Err() != nil
    # -> error (:440-443) -> PARSE_ERROR.
    body_m = struct.pack(">bb", 0, 0) + struct.pack(">i", 100) + b"k"
    import zlib
    msg = struct.pack(">I", zlib.crc32(body_m) & 0xFFFFFFFF) + body_m
    entry = struct.pack(">qi", 0, len(msg)) + msg
    body = struct.pack(">i", 1) + topic_hdr(T1, 1) + part_hdr(0, len(entry)) + entry
    out.append(("key past the message", produce_raw(body), True, PARSE_ERROR))
    return out


def classify(reqs, topic_rule):
    conns = gen.make_conns(1, 0, 9092, True, PROTO_KAFKA, [7], 9)
    arena, offs, lens = gen.pack(reqs)
    w = gen.Workload("wire", arena, offs, lens, np.zeros(len(reqs), np.uint32), conns, policy(topic_rule))
    return w


@pytest.mark.parametrize("name,req,topic_rule,want", cases(), ids=[c[0] for c in cases()])
def test_oracle_wire_kats(name, req, topic_rule, want):
    w = classify([req], topic_rule)
    v, r, c = refpy.classify_workload(w, 1)
    assert int(v[0]) == want, name
    if want in (ALLOW, DENY):
        assert int(c[0]) == len(req)


@pytest.mark.gpu
@pytest.mark.parametrize("topic_rule", [True, False])
def test_gpu_wire_kats(engine, oracle, topic_rule):
    from test_gpu_http import assert_same, both
    sel = [c for c in cases() if c[2] == topic_rule]
    w = classify([c[1] for c in sel], topic_rule)
    got, ref = both(engine, oracle, w, 1)
    assert_same(got, ref, w)
    assert got[0].tolist() == [c[3] for c in sel]
