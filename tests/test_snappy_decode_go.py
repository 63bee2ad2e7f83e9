"""Snappy block decoding pinned to the reference's vendored decoder.

The reference vendors github.com/golang/snappy (vendor/github.com/golang/
snappy/decode.go, decode_other.go; its amd64 assembly implements the same
contract) for optiopay's snappyDecode (proto/snappy.go).  Every vector below
is derived by hand from those lines: the input, and the output Decode returns
(None = an error).  The oracle's restatement (refpy.unsnappy) must agree with
each; tests/test_gpu_kafka_compressed.py::test_snappy_decode_go_vectors sends
the same inputs through the GPU inflate kernel inside produce requests.
"""
import pytest

import refpy


def uvarint(v):
    out = bytearray()
    while v >= 0x80:
        out.append((v & 0x7F) | 0x80)
        v >>= 7
    out.append(v)
    return bytes(out)


def lit(data):
    """a literal tag with a 1-byte-or-shorter length (x < 60)"""
    assert 0 < len(data) <= 60
    return bytes([(len(data) - 1) << 2]) + data


P70 = bytes(range(70))
P300 = bytes(i & 0xFF for i in range(300))
P70000 = bytes((i * 7) & 0xFF for i in range(70000))

# (name, src, expected, where in the reference the outcome is decided)
VECTORS = [
    ("empty input: no varint", b"", None, "decode.go:33-35 (n <= 0)"),
    ("unterminated varint", b"\x80", None, "decode.go:33-35 (n <= 0)"),
    ("decoded length > 0xffffffff", b"\x80\x80\x80\x80\x10", None, "decode.go:33-35 (v > 0xffffffff)"),
    ("empty block", b"\x00", b"", "decode.go:55-67; decode_other.go:16,97-100"),
    ("literal x < 60", uvarint(4) + lit(b"abcd"), b"abcd", "decode_other.go:19-22,48-58"),
    ("literal shorter than the block", uvarint(5) + lit(b"abcd"), None, "decode_other.go:97-98 (d != len(dst))"),
    ("literal x == 60", uvarint(70) + b"\xf0" + bytes([69]) + P70, P70, "decode_other.go:23-28"),
    ("literal x == 60, length byte missing", uvarint(70) + b"\xf0", None, "decode_other.go:25-26"),
    ("literal x == 61", uvarint(300) + b"\xf4" + (299).to_bytes(2, "little") + P300, P300, "decode_other.go:29-34"),
    ("literal x == 61, length bytes cut", uvarint(300) + b"\xf4\x2b", None, "decode_other.go:31-32"),
    ("literal x == 62", uvarint(70000) + b"\xf8" + (69999).to_bytes(3, "little") + P70000, P70000,
     "decode_other.go:35-40"),
    ("literal x == 63", uvarint(5) + b"\xfc" + (4).to_bytes(4, "little") + b"hello", b"hello", "decode_other.go:41-46"),
    ("literal x == 63, 2^32 bytes", uvarint(5) + b"\xfc\xff\xff\xff\xff" + b"hello", None,
     "decode_other.go:48-54 (length > len(dst)-d)"),
    ("literal past the input", uvarint(8) + bytes([7 << 2]) + b"abcd", None, "decode_other.go:52-54 (length > len(src)-s)"),
    ("literal past the block", uvarint(2) + lit(b"abcd"), None, "decode_other.go:52-54 (length > len(dst)-d)"),
    ("copy1", uvarint(8) + lit(b"abcd") + bytes([0x01, 4]), b"abcdabcd", "decode_other.go:60-66,85-95"),
    ("copy1 cut", uvarint(8) + lit(b"abcd") + bytes([0x01]), None, "decode_other.go:61-64"),
    ("copy1 offset 0", uvarint(8) + lit(b"abcd") + bytes([0x01, 0]), None, "decode_other.go:85-87 (offset <= 0)"),
    ("copy1 offset before the output", uvarint(8) + lit(b"abcd") + bytes([0x01, 5]), None,
     "decode_other.go:85-87 (d < offset)"),
    ("copy1 high offset bits", uvarint(4 + 4) + lit(b"abcd") + bytes([0x01 | (1 << 5), 4]), None,
     "decode_other.go:66,85-87 (offset = 0x104 > d)"),
    ("overlapping copy runs forwards", uvarint(8) + lit(b"ab") + bytes([((6 - 4) << 2) | 1, 2]), b"abababab",
     "decode_other.go:88-95"),
    ("copy past the block", uvarint(6) + lit(b"abcd") + bytes([0x01, 4]), None, "decode_other.go:85-87 (length > len(dst)-d)"),
    ("copy2", uvarint(8) + lit(b"abcd") + bytes([(3 << 2) | 2, 4, 0]), b"abcdabcd", "decode_other.go:68-74,85-95"),
    ("copy2 cut", uvarint(8) + lit(b"abcd") + bytes([(3 << 2) | 2, 4]), None, "decode_other.go:69-72"),
    ("copy2, 64-byte copy", uvarint(68) + lit(b"abcd") + bytes([(63 << 2) | 2, 4, 0]), b"abcd" * 17,
     "decode_other.go:73 (length = 1 + tag >> 2)"),
    ("copy4", uvarint(8) + lit(b"abcd") + bytes([(3 << 2) | 3, 4, 0, 0, 0]), b"abcdabcd", "decode_other.go:76-82,85-95"),
    ("copy4 cut", uvarint(8) + lit(b"abcd") + bytes([(3 << 2) | 3, 4, 0, 0]), None, "decode_other.go:77-80"),
    ("copy4 offset 2^32-1", uvarint(8) + lit(b"abcd") + bytes([(3 << 2) | 3, 0xFF, 0xFF, 0xFF, 0xFF]), None,
     "decode_other.go:85-87 (d < offset)"),
    ("trailing tag after a full block", uvarint(4) + lit(b"abcd") + bytes([0x01, 4]), None,
     "decode_other.go:85-87 (length > len(dst)-d)"),
]


@pytest.mark.parametrize("name,src,expected,where", VECTORS, ids=[v[0] for v in VECTORS])
def test_oracle_matches_vendored_decoder(name, src, expected, where):
    assert refpy.unsnappy(src) == expected, f"{name}: {where}"
