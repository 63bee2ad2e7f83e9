"""ctypes binding of include/l7gpu.h (the product's C-ABI).

The shared library is built in-tree by cilium_amd/build.py.  There is no
fallback: if libl7gpu.so is missing or fails to load, importing the engine
raises, so nothing can silently classify on the CPU.
"""
import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# L7G_LIB may name the profiling build (libl7gpu_timing.so) for experiments
LIB_PATH = os.environ.get("L7G_LIB") or os.path.join(HERE, "libl7gpu.so")

DENY, ALLOW, PARSE_ERROR, INCOMPLETE, UNSUPPORTED = 0, 1, 2, 3, 4
PROTO_HTTP, PROTO_KAFKA, PROTO_MEMCACHE, PROTO_R2D2, PROTO_CASSANDRA = 1, 2, 3, 4, 5
VERDICT_NAMES = {DENY: "DENY", ALLOW: "ALLOW", PARSE_ERROR: "PARSE_ERROR",
                 INCOMPLETE: "INCOMPLETE", UNSUPPORTED: "UNSUPPORTED"}


class Conn(C.Structure):
    """l7g_conn_t (20 bytes; same layout as the oracle's ref_conn_t)."""
    _fields_ = [("policy", C.c_int32), ("port", C.c_uint32), ("ingress", C.c_uint8),
                ("proto", C.c_uint8), ("flags", C.c_uint16), ("src_id", C.c_uint32),
                ("dst_id", C.c_uint32)]


class Stats(C.Structure):
    _fields_ = [(n, C.c_uint32) for n in (
        "policies", "rules", "http_rulesets", "http_chunks", "http_dfas", "http_dfa_states",
        "kafka_rulesets", "kafka_rules", "kafka_topics")] + [
        ("table_bytes", C.c_uint64), ("http_image_bytes", C.c_uint64), ("hot_ruleset", C.c_int32),
        ("hot_image_bytes", C.c_uint32)] + [
        (n, C.c_uint32) for n in ("mc_rulesets", "mc_rules", "mc_dfas", "mc_dfa_states", "http_nfas", "mc_nfas")] + [
        ("nfa_pool_bytes", C.c_uint64), ("r2d2_rulesets", C.c_uint32), ("r2d2_rules", C.c_uint32)]


EXPORTS = (
    "l7g_engine_create", "l7g_engine_destroy", "l7g_policy_update", "l7g_policy_index",
    "l7g_policy_nrules", "l7g_conns_set", "l7g_conn_update", "l7g_classify", "l7g_classify_host", "l7g_stats",
    "l7g_debug_regex", "l7g_debug_phase_times", "l7g_profile_enable", "l7g_profile_last",
    "l7g_debug_kafka_phase_times", "l7g_debug_frame_phase_times", "l7g_kafka_deny_response", "l7g_debug_regex_nfa", "l7g_policy_update_proto", "l7g_kafka_corr_create", "l7g_kafka_corr_destroy",
    "l7g_kafka_corr_requests", "l7g_kafka_corr_responses", "l7g_kafka_corr_gc", "l7g_kafka_corr_size",
    "l7g_flow_stats_enable", "l7g_flow_stats",
    "l7g_tables_export", "l7g_tables_import", "l7g_tables_compiled", "l7g_tables_digest",
    "l7g_frame_streams", "l7g_classify_streams", "l7g_service_enable", "l7g_service_stats",
)


class FlowStat(C.Structure):
    _fields_ = [("policy", C.c_int32), ("proto", C.c_uint8), ("ingress", C.c_uint8), ("port", C.c_uint16),
                ("received", C.c_uint64), ("forwarded", C.c_uint64), ("denied", C.c_uint64), ("error", C.c_uint64)]

_libs = {}


def load(path=None):
    """The product library (or, for kernel experiments, a variant build of it
    named by path: tools/exp_*.py)."""
    path = path or LIB_PATH
    if path in _libs:
        return _libs[path]
    if not os.path.exists(path):
        raise RuntimeError(f"{path} is missing: run python -m cilium_amd.build (no CPU fallback exists)")
    # One HIP runtime per process: torch ships its own libamdhip64 under the same
    # soname, and whichever loads first serves both.  Loading torch's first keeps
    # torch.cuda working in processes that use both (batches in torch tensors).
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    lib = C.CDLL(path)
    vp, sz, cp = C.c_void_p, C.c_size_t, C.c_char_p
    lib.l7g_engine_create.restype = vp
    lib.l7g_engine_create.argtypes = [C.c_int, cp, sz]
    lib.l7g_engine_destroy.argtypes = [vp]
    lib.l7g_policy_update.argtypes = [vp, cp, sz, cp, sz]
    lib.l7g_policy_update_proto.argtypes = [vp, cp, sz, cp, sz]
    lib.l7g_policy_index.restype = C.c_int32
    lib.l7g_policy_index.argtypes = [vp, cp, sz]
    lib.l7g_policy_nrules.restype = C.c_int32
    lib.l7g_policy_nrules.argtypes = [vp]
    lib.l7g_conns_set.argtypes = [vp, vp, C.c_uint32, cp, sz]
    lib.l7g_tables_export.argtypes = [vp, vp, sz, C.POINTER(sz)]
    lib.l7g_tables_import.argtypes = [vp, cp, sz, cp, sz]
    lib.l7g_tables_compiled.restype = C.c_uint64
    lib.l7g_tables_compiled.argtypes = [vp]
    lib.l7g_tables_digest.restype = C.c_uint64
    lib.l7g_tables_digest.argtypes = [vp]
    lib.l7g_conn_update.argtypes = [vp, C.c_uint32, vp, cp, sz]
    lib.l7g_classify.argtypes = [vp, vp, C.c_uint64, vp, vp, vp, C.c_uint32, vp, vp, vp, vp, vp]
    lib.l7g_frame_streams.argtypes = [vp, vp, C.c_uint64, vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp]
    lib.l7g_classify_streams.argtypes = [vp, vp, C.c_uint64, vp, vp, vp, C.c_uint32, C.c_uint32, vp, vp, vp, vp, vp, vp,
                                         vp, vp, vp]
    lib.l7g_classify_host.argtypes = [vp, vp, C.c_uint64, vp, vp, vp, C.c_uint32, vp, vp, vp]
    lib.l7g_service_enable.argtypes = [vp, C.c_int]
    lib.l7g_service_stats.argtypes = [vp, C.POINTER(C.c_uint64)]
    lib.l7g_service_stats.restype = None
    lib.l7g_stats.argtypes = [vp, C.POINTER(Stats)]
    lib.l7g_debug_regex.argtypes = [cp, sz, C.c_int, cp, sz, cp, sz]
    lib.l7g_debug_regex_nfa.argtypes = [cp, sz, C.c_int, cp, sz, cp, sz]
    lib.l7g_debug_phase_times.argtypes = [vp, vp, C.c_int]
    lib.l7g_debug_kafka_phase_times.argtypes = [vp, vp, C.c_int]
    lib.l7g_debug_frame_phase_times.argtypes = [vp, vp, C.c_int]
    lib.l7g_kafka_corr_create.restype = vp
    lib.l7g_kafka_corr_destroy.argtypes = [vp]
    lib.l7g_kafka_corr_requests.argtypes = [vp, vp, vp, vp, C.c_uint32, vp]
    lib.l7g_kafka_corr_responses.argtypes = [vp, vp, vp, vp, C.c_uint32, vp]
    lib.l7g_kafka_corr_gc.restype = C.c_uint64
    lib.l7g_kafka_corr_gc.argtypes = [vp, C.c_uint64]
    lib.l7g_kafka_corr_size.restype = C.c_uint64
    lib.l7g_kafka_corr_size.argtypes = [vp]
    lib.l7g_kafka_deny_response.argtypes = [cp, sz, vp, sz, C.POINTER(C.c_size_t)]
    lib.l7g_profile_enable.argtypes = [vp, C.c_int]
    lib.l7g_flow_stats_enable.argtypes = [vp, C.c_int]
    lib.l7g_flow_stats.argtypes = [vp, vp, C.c_uint32, C.POINTER(C.c_uint32), C.c_int]
    lib.l7g_profile_last.argtypes = [vp, vp]
    _libs[path] = lib
    return lib


def debug_regex(pattern, data, anchored=True, nfa=False):
    """Compile `pattern` with the product's Go-regexp DFA compiler (nfa=True:
    the bit-parallel NFA fallback) and run the compiled tables on `data` (host
    walk of the device tables; test hook).  Returns True/False, or raises
    ValueError with Go's compile error text."""
    lib = load()
    p = pattern.encode() if isinstance(pattern, str) else pattern
    d = data.encode() if isinstance(data, str) else data
    err = C.create_string_buffer(512)
    fn = lib.l7g_debug_regex_nfa if nfa else lib.l7g_debug_regex
    r = fn(p, len(p), 1 if anchored else 0, d, len(d), err, 512)
    if r < 0:
        raise ValueError(err.value.decode(errors="replace"))
    return bool(r)


def kafka_deny_response(req):
    """The bytes the Kafka proxy answers a denied request with
    (CreateResponse(ErrTopicAuthorizationFailed)), or None (untyped kind /
    undecodable request: no response)."""
    lib = load()
    cap = 4 * len(req) + 256
    out = C.create_string_buffer(cap)
    n = C.c_size_t(0)
    rc = lib.l7g_kafka_deny_response(req, len(req), out, cap, C.byref(n))
    if rc == -1:
        return None
    if rc != 0:
        raise RuntimeError(f"l7g_kafka_deny_response: {rc}")
    return out.raw[:n.value]


class KafkaCorrelationCache:
    """One client connection's correlation cache (l7g_kafka_corr_*): batches
    of frames given as (arena: writable uint8 numpy array, offsets, lengths)."""

    def __init__(self):
        self._lib = load()
        self._h = self._lib.l7g_kafka_corr_create()

    def __del__(self):
        try:
            self._lib.l7g_kafka_corr_destroy(self._h)
        except Exception:
            pass

    def requests(self, arena, offs, lens):
        import numpy as np
        o = np.ascontiguousarray(offs, np.uint64)
        n = np.ascontiguousarray(lens, np.uint32)
        ids = np.zeros(len(o), np.uint32)
        self._lib.l7g_kafka_corr_requests(self._h, arena.ctypes.data, o.ctypes.data, n.ctypes.data, len(o), ids.ctypes.data)
        return ids

    def responses(self, arena, offs, lens):
        import numpy as np
        o = np.ascontiguousarray(offs, np.uint64)
        n = np.ascontiguousarray(lens, np.uint32)
        found = np.zeros(len(o), np.uint8)
        self._lib.l7g_kafka_corr_responses(self._h, arena.ctypes.data, o.ctypes.data, n.ctypes.data, len(o),
                                           found.ctypes.data)
        return found.astype(bool)

    def gc(self, lifetime_ms):
        return int(self._lib.l7g_kafka_corr_gc(self._h, lifetime_ms))

    def __len__(self):
        return int(self._lib.l7g_kafka_corr_size(self._h))
