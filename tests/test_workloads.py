"""Host-side checks of the bench workloads (no GPU): the cfg5 mixed stream,
device tiling offsets and the memcached inspected-byte accounting used for
roofline.achieved."""
import struct

import numpy as np

from cilium_amd import gen
from cilium_amd._lib import PROTO_HTTP, PROTO_KAFKA, PROTO_MEMCACHE


def test_mixed_workload_shape_and_oracle():
    import refpy
    w = gen.mixed_workload(3000)
    assert w.n == 3000
    proto = w.conns["proto"][w.conn_ids]
    assert (proto == PROTO_HTTP).sum() == 1500
    assert (proto == PROTO_KAFKA).sum() == 900
    assert (proto == PROTO_MEMCACHE).sum() == 600
    # repacked in arrival order: offsets strictly follow one another
    assert np.array_equal(w.offsets[1:], w.offsets[:-1] + w.lengths[:-1].astype(np.uint64))
    refpy.build()
    v, r, c = refpy.Policy(w.policy).classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids, 4)
    hist = np.bincount(v, minlength=5)
    assert hist[0] > 0 and hist[1] > 0  # both allow and deny occur
    assert (c[v == 1] > 0).all()


def test_tile_offsets():
    w = gen.http_workload(2, 50)
    offs, lens, cids = gen.tile_offsets(w, 4)
    assert len(offs) == 200
    for j in range(4):
        assert np.array_equal(offs[j * 50:(j + 1) * 50], w.offsets + np.uint64(j * len(w.arena)))
    assert np.array_equal(lens, np.tile(w.lengths, 4)) and np.array_equal(cids, np.tile(w.conn_ids, 4))
    o1, l1, c1 = gen.tile_offsets(w, 1)
    assert o1 is w.offsets


def test_mc_inspected_bytes():
    text_set = b"set k 0 0 5\r\nhello\r\n"
    text_get = b"get a b\r\n"
    binary = gen.mc_bin(1, b"key", bytes(8), b"value-bytes")
    assert struct.unpack(">H", binary[2:4])[0] == 3
    assert gen.mc_inspected_bytes([text_set]) == len(b"set k 0 0 5\r\n")
    assert gen.mc_inspected_bytes([text_get]) == len(text_get)
    assert gen.mc_inspected_bytes([binary]) == 24 + 8 + 3
    assert gen.mc_inspected_bytes([b"get a"]) == 5  # no CRLF: the whole buffer is inspected
    w = gen.memcache_workload(500)
    assert w.algorithmic_bytes() < int(w.lengths.astype(np.int64).sum()) + 25 * w.n
