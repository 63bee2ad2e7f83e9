"""Host-side engine: the Python face of the C-ABI (include/l7gpu.h).

Mirrors the reference's per-request verdict interface for this path:
policies in (NPDS cilium.NetworkPolicy shape), connections opened with their
(policy, port, direction, identities) as in proxylib OnNewConnection
(proxylib/proxylib.go:57-74), then batches of requests classified into
(verdict, matched rule, consumed bytes).
"""
import ctypes as C
import json

import numpy as np

from . import _lib
from ._lib import Conn


class PolicyError(ValueError):
    """The policy set was rejected (the reference would NACK it)."""


class Engine:
    def __init__(self, device=0, lib_path=None):
        self._lib = _lib.load(lib_path)
        err = C.create_string_buffer(512)
        h = self._lib.l7g_engine_create(device, err, 512)
        if not h:
            raise RuntimeError("l7g_engine_create: " + err.value.decode(errors="replace"))
        self._h = h
        self.device = device

    def close(self):
        if getattr(self, "_h", None):
            self._lib.l7g_engine_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    # ---------------------------------------------------------------- policy
    def update_policy(self, policy):
        js = policy if isinstance(policy, (str, bytes)) else json.dumps(policy)
        b = js.encode() if isinstance(js, str) else js
        err = C.create_string_buffer(1024)
        if self._lib.l7g_policy_update(self._h, b, len(b), err, 1024) != 0:
            raise PolicyError(err.value.decode(errors="replace"))

    def update_policy_proto(self, buf):
        """A serialized NPDS DiscoveryResponse (cilium.NetworkPolicy resources)."""
        b = bytes(buf)
        err = C.create_string_buffer(1024)
        if self._lib.l7g_policy_update_proto(self._h, b, len(b), err, 1024) != 0:
            raise PolicyError(err.value.decode(errors="replace"))

    def export_tables(self):
        """The current policy version's compiled tables (l7g_tables_export):
        what rank 0 broadcasts so that the other ranks install them without
        compiling (cilium_amd/dist.py)."""
        n = C.c_size_t(0)
        self._lib.l7g_tables_export(self._h, None, 0, C.byref(n))
        buf = (C.c_uint8 * max(n.value, 1))()
        if self._lib.l7g_tables_export(self._h, buf, n.value, C.byref(n)) != 0:
            raise RuntimeError("l7g_tables_export failed")
        return bytes(buf)[:n.value]

    def import_tables(self, image):
        b = bytes(image)
        err = C.create_string_buffer(1024)
        if self._lib.l7g_tables_import(self._h, b, len(b), err, 1024) != 0:
            raise PolicyError(err.value.decode(errors="replace"))

    @property
    def tables_compiled(self):
        """Rule sets this engine compiled itself since its policy version was installed."""
        return int(self._lib.l7g_tables_compiled(self._h))

    @property
    def tables_digest(self):
        """FNV-1a 64 of the device table blob (equal <=> byte-identical tables)."""
        return int(self._lib.l7g_tables_digest(self._h))

    def policy_index(self, name):
        b = name.encode()
        return self._lib.l7g_policy_index(self._h, b, len(b))

    @property
    def nrules(self):
        return self._lib.l7g_policy_nrules(self._h)

    # ----------------------------------------------------------- connections
    def set_connections(self, conns):
        """conns: sequence of dicts/tuples (policy, port, ingress, proto, src_id, dst_id)
        or a numpy structured array with those fields."""
        arr = conns_array(conns)
        err = C.create_string_buffer(1024)
        if self._lib.l7g_conns_set(self._h, arr.ctypes.data, len(arr), err, 1024) != 0:
            raise PolicyError(err.value.decode(errors="replace"))
        self._conns = arr

    # --------------------------------------------------------- classification
    def classify_device(self, arena_ptr, arena_len, off_ptr, len_ptr, conn_ptr, n, verdict_ptr, rule_ptr,
                        consumed_ptr, counters_ptr=0, stream=0):
        """All pointers are device addresses (e.g. torch tensor .data_ptr());
        every request lies inside [arena_ptr, arena_ptr + arena_len)."""
        rc = self._lib.l7g_classify(self._h, arena_ptr, arena_len, off_ptr, len_ptr, conn_ptr, n, verdict_ptr,
                                    rule_ptr, consumed_ptr, counters_ptr or None, stream or None)
        if rc != 0:
            raise RuntimeError(f"l7g_classify failed: HIP error {rc}")

    def classify_streams_device(self, arena_ptr, arena_len, s_off_ptr, s_len_ptr, s_conn_ptr, n, max_frames,
                                frame_off_ptr, frame_len_ptr, frame_conn_ptr, nframes_ptr, verdict_ptr=0, rule_ptr=0,
                                consumed_ptr=0, counters_ptr=0, stream=0):
        """l7g_frame_streams (no verdict pointers) or l7g_classify_streams: device
        framing of n connection streams into n * max_frames frame slots."""
        if verdict_ptr:
            rc = self._lib.l7g_classify_streams(self._h, arena_ptr, arena_len, s_off_ptr, s_len_ptr, s_conn_ptr, n,
                                                max_frames, frame_off_ptr, frame_len_ptr, frame_conn_ptr, nframes_ptr,
                                                verdict_ptr, rule_ptr, consumed_ptr, counters_ptr or None,
                                                stream or None)
        else:
            rc = self._lib.l7g_frame_streams(self._h, arena_ptr, arena_len, s_off_ptr, s_len_ptr, s_conn_ptr, n,
                                             max_frames, frame_off_ptr, frame_len_ptr, frame_conn_ptr, nframes_ptr,
                                             stream or None)
        if rc != 0:
            raise RuntimeError(f"l7g_frame_streams / l7g_classify_streams failed: HIP error {rc}")

    def classify(self, arena, offsets, lengths, conn_ids):
        """Host-buffer convenience: copies to the device, classifies, copies back."""
        arena = np.ascontiguousarray(arena, dtype=np.uint8)
        off = np.ascontiguousarray(offsets, dtype=np.uint64)
        ln = np.ascontiguousarray(lengths, dtype=np.uint32)
        cid = np.ascontiguousarray(conn_ids, dtype=np.uint32)
        n = len(off)
        v = np.zeros(n, np.uint8)
        r = np.zeros(n, np.int32)
        c = np.zeros(n, np.uint32)
        rc = self._lib.l7g_classify_host(self._h, arena.ctypes.data, arena.nbytes, off.ctypes.data,
                                         ln.ctypes.data, cid.ctypes.data, n, v.ctypes.data,
                                         r.ctypes.data, c.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"l7g_classify_host failed: HIP error {rc}")
        return v, r, c

    STAGES = ("partition", "http", "kafka", "memcache")

    def profile(self, on=True):
        """Record HIP events around each kernel of every l7g_classify call."""
        rc = self._lib.l7g_profile_enable(self._h, 1 if on else 0)
        if rc != 0:
            raise RuntimeError(f"l7g_profile_enable failed: HIP error {rc}")

    def profile_last(self):
        """Device ms per stage of the last classify call (profiling on)."""
        out = np.zeros(4, np.float32)
        rc = self._lib.l7g_profile_last(self._h, out.ctypes.data)
        if rc != 0:
            raise RuntimeError(f"l7g_profile_last failed: HIP error {rc}")
        return dict(zip(self.STAGES, out.tolist()))

    def kafka_phase_times(self, reset=True):
        """Per-phase cycle totals of the Kafka kernel (-DL7G_KX_TIMING build only), or None."""
        out = np.zeros(8, np.uint64)
        if self._lib.l7g_debug_kafka_phase_times(self._h, out.ctypes.data, 1 if reset else 0) != 0:
            return None
        return out

    def frame_phase_times(self, reset=True):
        """Per-phase cycle totals of the text-stream framer (-DL7G_FRAME_PHASES build only), or None."""
        out = np.zeros(8, np.uint64)
        if self._lib.l7g_debug_frame_phase_times(self._h, out.ctypes.data, 1 if reset else 0) != 0:
            return None
        return out

    def phase_times(self, reset=True):
        """Per-phase cycle totals of the HTTP kernels (timing build only; 16 slots,
        include/l7gpu.h), or None."""
        out = np.zeros(16, np.uint64)
        if self._lib.l7g_debug_phase_times(self._h, out.ctypes.data, 1 if reset else 0) != 0:
            return None
        return out

    def flow_stats_enable(self, on=True):
        rc = self._lib.l7g_flow_stats_enable(self._h, 1 if on else 0)
        if rc != 0:
            raise RuntimeError(f"l7g_flow_stats_enable: {rc}")

    def flow_stats(self, reset=False):
        """{(policy, proto, port, ingress): (received, forwarded, denied, error)}
        accumulated since the last reset (pkg/endpoint UpdateProxyStatistics)."""
        n = C.c_uint32(0)
        rc = self._lib.l7g_flow_stats(self._h, None, 0, C.byref(n), 0)
        if rc != 0:
            raise RuntimeError(f"l7g_flow_stats: {rc}")
        arr = (_lib.FlowStat * max(1, n.value))()
        rc = self._lib.l7g_flow_stats(self._h, arr, n.value, C.byref(n), 1 if reset else 0)
        if rc != 0:
            raise RuntimeError(f"l7g_flow_stats: {rc}")
        return {(x.policy, x.proto, x.port, x.ingress): (x.received, x.forwarded, x.denied, x.error)
                for x in arr[:n.value]}

    def service(self, on=None):
        """Resident services (l7g_service_enable): with on given, enable (True)
        or stop and disable (False); returns the previous setting and the
        counts {http_calls, http_launches, mc_calls, mc_launches}."""
        prev = None
        if on is not None:
            prev = bool(self._lib.l7g_service_enable(self._h, 1 if on else 0))
        out = (C.c_uint64 * 4)()
        self._lib.l7g_service_stats(self._h, out)
        return prev, dict(zip(("http_calls", "http_launches", "mc_calls", "mc_launches"), list(out)))

    def stats(self):
        s = _lib.Stats()
        self._lib.l7g_stats(self._h, C.byref(s))
        return {k: getattr(s, k) for k, _ in s._fields_}


CONN_DTYPE = np.dtype([("policy", "<i4"), ("port", "<u4"), ("ingress", "u1"), ("proto", "u1"),
                       ("flags", "<u2"), ("src_id", "<u4"), ("dst_id", "<u4")])
assert CONN_DTYPE.itemsize == C.sizeof(Conn)


def conns_array(conns):
    if isinstance(conns, np.ndarray) and conns.dtype == CONN_DTYPE:
        return np.ascontiguousarray(conns)
    arr = np.zeros(len(conns), CONN_DTYPE)
    for i, c in enumerate(conns):
        if isinstance(c, dict):
            for k in ("policy", "port", "ingress", "proto", "flags", "src_id", "dst_id"):
                arr[i][k] = c.get(k, 0)
        else:
            arr[i] = (c[0], c[1], c[2], c[3], 0, c[4], c[5])
    return arr
