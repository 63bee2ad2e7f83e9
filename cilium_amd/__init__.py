"""cilium_amd — MI355X-native batched L7 policy classifier for Cilium's
HTTP / Kafka request-filtering path.

The product is the C-ABI shared library libl7gpu.so (HIP kernels for gfx950 +
C++ rule compiler).  This package is its Python face: ctypes bindings, the
rule-model mirror of pkg/policy/api (api.py) and the synthetic workload
generators used by tests and bench.py (gen.py).
"""
from ._lib import (ALLOW, DENY, INCOMPLETE, PARSE_ERROR, PROTO_HTTP, PROTO_KAFKA,  # noqa: F401
                   PROTO_MEMCACHE, UNSUPPORTED, VERDICT_NAMES, debug_regex)
from .engine import CONN_DTYPE, Engine, PolicyError, conns_array  # noqa: F401
