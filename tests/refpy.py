"""ctypes wrapper of the parity oracle (oracle/build/libl7ref.so).

TEST INFRASTRUCTURE ONLY: used by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker / CPU baseline, never as the
product path.
"""
import ctypes as C
import json
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
LIB = os.path.join(ORACLE_DIR, "build", "libl7ref.so")

_lib = None


def build():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return LIB


def load():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        lib = C.CDLL(LIB)
        vp, sz, cp = C.c_void_p, C.c_size_t, C.c_char_p
        lib.ref_re_compile.restype = vp
        lib.ref_re_compile.argtypes = [cp, sz, cp, sz]
        lib.ref_re_free.argtypes = [vp]
        lib.ref_re_match.argtypes = [vp, cp, sz, C.c_int]
        lib.ref_policy_load.restype = vp
        lib.ref_policy_load.argtypes = [cp, sz, cp, sz]
        lib.ref_policy_free.argtypes = [vp]
        lib.ref_classify.argtypes = [vp, vp, C.c_uint32, vp, vp, vp, vp, C.c_uint32, vp, vp, vp, C.c_int]
        for f in (lib.ref_gunzip, lib.ref_unsnappy):
            f.argtypes = [cp, sz, vp, sz, C.POINTER(sz)]
        lib.ref_cass_new.restype = vp
        lib.ref_cass_free.argtypes = [vp]
        lib.ref_cass_request.argtypes = [vp, vp, vp, cp, C.c_uint32, C.POINTER(C.c_int64), C.POINTER(C.c_int32),
                                         C.POINTER(vp), vp, C.POINTER(C.c_uint32)]
        lib.ref_cass_reply.argtypes = [vp, cp, C.c_uint32, C.POINTER(C.c_int64)]
        lib.ref_cass_parse_query.argtypes = [vp, cp, sz, cp, sz, cp, sz]
        lib.ref_cass_keyspace.restype = cp
        lib.ref_cass_keyspace.argtypes = [vp]
        _lib = lib
    return _lib


class Regex:
    def __init__(self, pattern):
        lib = load()
        b = pattern.encode() if isinstance(pattern, str) else pattern
        err = C.create_string_buffer(512)
        self._h = lib.ref_re_compile(b, len(b), err, 512)
        if not self._h:
            raise ValueError(err.value.decode(errors="replace"))

    def match(self, data, anchored=True):
        d = data.encode() if isinstance(data, str) else data
        return bool(load().ref_re_match(self._h, d, len(d), 1 if anchored else 0))

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ref_re_free(self._h)


class Policy:
    def __init__(self, policy):
        lib = load()
        js = policy if isinstance(policy, (str, bytes)) else json.dumps(policy)
        b = js.encode() if isinstance(js, str) else js
        err = C.create_string_buffer(1024)
        self._h = lib.ref_policy_load(b, len(b), err, 1024)
        if not self._h:
            raise ValueError(err.value.decode(errors="replace"))
        self.names = {}
        obj = json.loads(b)
        for i, p in enumerate(obj["policies"] if isinstance(obj, dict) else obj):
            self.names.setdefault(p.get("name", ""), i)

    def classify(self, conns, arena, offsets, lengths, conn_ids, nthreads=1):
        lib = load()
        from cilium_amd.engine import conns_array
        conns = conns_array(conns)
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        cid = np.ascontiguousarray(conn_ids, dtype=np.uint32)
        n = len(off)
        v = np.zeros(n, np.uint8)
        r = np.zeros(n, np.int32)
        c = np.zeros(n, np.uint32)
        lib.ref_classify(self._h, conns.ctypes.data, len(conns), arena.ctypes.data, off.ctypes.data,
                         ln.ctypes.data, cid.ctypes.data, n, v.ctypes.data, r.ctypes.data, c.ctypes.data,
                         nthreads)
        return v, r, c

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.ref_policy_free(self._h)


MAX_PARSE_BUF = 6_553_500


def _decode(fn, data, cap):
    out = C.create_string_buffer(max(cap, 1))
    n = C.c_size_t(0)
    if fn(data, len(data), out, cap, C.byref(n)) != 0:
        return None
    return out.raw[:n.value]


def gunzip(data, cap=MAX_PARSE_BUF):
    """Go's gzip.NewReader + ReadAll restated (oracle/kafka_inflate.c): the
    decoded bytes, or None on any error / more than cap bytes."""
    return _decode(load().ref_gunzip, data, cap)


def unsnappy(data, cap=MAX_PARSE_BUF):
    """proto.snappyDecode restated (plain snappy or xerial framing)."""
    return _decode(load().ref_unsnappy, data, cap)


def classify_workload(w, nthreads=1):
    return Policy(w.policy).classify(w.conns, w.arena, w.offsets, w.lengths, w.conn_ids, nthreads)


class Cassandra:
    """One proxylib cassandra parser state (oracle/cassandra_ref.c): keyspace of
    the last USE and the prepared-statement paths."""
    PANIC = -1

    def __init__(self, policy=None, conn=None):
        self._lib = load()
        self._h = self._lib.ref_cass_new()
        self.policy = policy  # refpy.Policy
        self.conn = conn      # one CONN_DTYPE record

    def __del__(self):
        if getattr(self, "_h", None):
            self._lib.ref_cass_free(self._h)

    def parse_query(self, q):
        """(status, action, table): status 0 ok, 1 invalid, 2 panic."""
        b = q.encode() if isinstance(q, str) else q
        a, t = C.create_string_buffer(1 << 16), C.create_string_buffer(1 << 16)
        rc = self._lib.ref_cass_parse_query(self._h, b, len(b), a, len(a), t, len(t))
        return rc, a.value, t.value

    @property
    def keyspace(self):
        return self._lib.ref_cass_keyspace(self._h)

    def request(self, data):
        """One request-direction OnData step: (op, n, rule, path, inject)."""
        from cilium_amd.engine import conns_array
        c = conns_array([self.conn]) if not isinstance(self.conn, np.ndarray) else self.conn
        n, rule = C.c_int64(0), C.c_int32(0)
        path = C.c_void_p(0)
        inj = C.create_string_buffer(65600)
        il = C.c_uint32(0)
        op = self._lib.ref_cass_request(self._h, self.policy._h, c.ctypes.data, data, len(data), C.byref(n),
                                        C.byref(rule), C.byref(path), inj, C.byref(il))
        p = C.string_at(path.value) if path.value else None
        if path.value:
            C.CDLL(None).free(path)
        return op, n.value, rule.value, p, inj.raw[:il.value]

    def reply(self, data):
        n = C.c_int64(0)
        op = self._lib.ref_cass_reply(self._h, data, len(data), C.byref(n))
        return op, n.value
