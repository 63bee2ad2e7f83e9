"""ctypes view of the proxylib C-ABI that libl7gpu.so exports
(include/proxylib_abi.h; the reference's proxylib/libcilium.h:13-115 types).

This is how a cgo / Envoy caller sees the library: GoString / GoSlice
arguments, caller-owned inject buffers and op arrays.  The tests drive it the
way proxylib's own Go tests drive OpenModule / OnNewConnection / OnData
(proxylib/helpers_test.go:52-144).
"""
import ctypes as C
import json

from . import _lib

MORE, PASS, DROP, INJECT, ERROR = 0, 1, 2, 3, 4
OK, POLICY_DROP, PARSER_ERROR, UNKNOWN_PARSER, UNKNOWN_CONNECTION, INVALID_ADDRESS, INVALID_INSTANCE, \
    UNKNOWN_ERROR = range(8)


class GoString(C.Structure):
    _fields_ = [("p", C.c_char_p), ("n", C.c_ssize_t)]


class GoSlice(C.Structure):
    _fields_ = [("data", C.c_void_p), ("len", C.c_int64), ("cap", C.c_int64)]


def gostr(s):
    b = s.encode() if isinstance(s, str) else s
    return GoString(b, len(b))


_bound = None


def lib():
    global _bound
    if _bound is None:
        L = _lib.load()
        L.OpenModule.restype = C.c_uint64
        L.OpenModule.argtypes = [GoSlice, C.c_uint8]
        L.CloseModule.argtypes = [C.c_uint64]
        L.OnNewConnection.restype = C.c_int
        L.OnNewConnection.argtypes = [C.c_uint64, GoString, C.c_uint64, C.c_uint8, C.c_uint32, C.c_uint32, GoString,
                                      GoString, GoString, C.POINTER(GoSlice), C.POINTER(GoSlice)]
        L.OnData.restype = C.c_int
        L.OnData.argtypes = [C.c_uint64, C.c_uint8, C.c_uint8, C.POINTER(GoSlice), C.POINTER(GoSlice)]
        L.Close.argtypes = [C.c_uint64]
        L.l7g_proxylib_policy_update.restype = C.c_int
        L.l7g_proxylib_policy_update.argtypes = [C.c_uint64, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.l7g_proxylib_policy_update_proto.restype = C.c_int
        L.l7g_proxylib_policy_update_proto.argtypes = [C.c_uint64, C.c_char_p, C.c_size_t, C.c_char_p, C.c_size_t]
        L.l7g_proxylib_connections.restype = C.c_uint64
        _bound = L
    return _bound


def open_module(params=(), debug=False):
    """params: sequence of (key, value); returns the instance id (0 = error)."""
    keep = [(gostr(k), gostr(v)) for k, v in params]
    arr = (GoString * (2 * max(1, len(keep))))()
    for i, (k, v) in enumerate(keep):
        arr[2 * i], arr[2 * i + 1] = k, v
    return lib().OpenModule(GoSlice(C.cast(arr, C.c_void_p), len(keep), len(keep)), 1 if debug else 0)


def close_module(mid):
    lib().CloseModule(mid)


def policy_update(mid, policy):
    js = policy if isinstance(policy, (str, bytes)) else json.dumps(policy)
    b = js.encode() if isinstance(js, str) else js
    err = C.create_string_buffer(1024)
    if lib().l7g_proxylib_policy_update(mid, b, len(b), err, 1024) != 0:
        raise ValueError(err.value.decode(errors="replace"))


def connections():
    return int(lib().l7g_proxylib_connections())


class Connection:
    """A caller-side connection: owns the two inject buffers (fixed capacity,
    never reallocated) for as long as the connection is open."""

    def __init__(self, mid, proto, conn_id, ingress, src_id, dst_id, src_addr, dst_addr, policy_name, buf_size=1024):
        self.id = conn_id
        self._orig_mem = (C.c_uint8 * buf_size)()
        self._reply_mem = (C.c_uint8 * buf_size)()
        self.orig = GoSlice(C.cast(self._orig_mem, C.c_void_p), 0, buf_size)
        self.reply = GoSlice(C.cast(self._reply_mem, C.c_void_p), 0, buf_size)
        self.result = lib().OnNewConnection(mid, gostr(proto), conn_id, 1 if ingress else 0, src_id, dst_id,
                                            gostr(src_addr), gostr(dst_addr), gostr(policy_name),
                                            C.byref(self.orig), C.byref(self.reply))

    def on_data(self, reply, buffers, max_ops, end_stream=False):
        """Returns (FilterResult, [(op, n), ...])."""
        return on_data(self.id, reply, buffers, max_ops, end_stream)

    def take_inject(self, reply=True):
        s = self.reply if reply else self.orig
        mem = self._reply_mem if reply else self._orig_mem
        out = bytes(mem[:s.len])
        s.len = 0
        return out

    def close(self):
        lib().Close(self.id)


def on_data(conn_id, reply, buffers, max_ops, end_stream=False):
    keep = [C.create_string_buffer(bytes(b), len(b)) for b in buffers]
    slices = (GoSlice * max(1, len(keep)))()
    for i, b in enumerate(keep):
        slices[i] = GoSlice(C.cast(b, C.c_void_p), len(b), len(b))
    data = GoSlice(C.cast(slices, C.c_void_p), len(keep), len(keep))
    ops_mem = (C.c_int64 * (2 * max(1, max_ops)))()
    ops = GoSlice(C.cast(ops_mem, C.c_void_p), 0, max_ops)
    res = lib().OnData(conn_id, 1 if reply else 0, 1 if end_stream else 0, C.byref(data), C.byref(ops))
    return res, [(int(ops_mem[2 * i]), int(ops_mem[2 * i + 1])) for i in range(ops.len)]


def policy_update_proto(mid, buf):
    """NPDS wire form: a serialized DiscoveryResponse of cilium.NetworkPolicy."""
    b = bytes(buf)
    err = C.create_string_buffer(1024)
    if lib().l7g_proxylib_policy_update_proto(mid, b, len(b), err, 1024) != 0:
        raise ValueError(err.value.decode(errors="replace"))
