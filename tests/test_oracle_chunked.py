"""The oracle's chunked-body contract on hand-derived cases.

Envoy's HTTP/1 codec at the pinned commit (envoy/WORKSPACE:10, http_parser)
frames a request with Transfer-Encoding: chunked by its chunks; the
cilium.l7policy filter decides on the headers alone
(envoy/cilium_l7policy.cc:127-182).  No reference test covers this: the
expected values below are derived by hand from the contract (parity unpinned).
"""
import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, DENY, INCOMPLETE, PARSE_ERROR

HEAD = b"GET /public/abc/7/x HTTP/1.1\r\nHost: svc-7.q\r\n"


def run(oracle, reqs):
    pol = gen.cfg1_policy()  # GET /public/.* => ALLOW
    w = gen.Workload("t", *gen.pack(reqs), np.zeros(len(reqs), np.uint32),
                     gen.make_conns(1, 0, 80, True, 1, [1]), pol)
    return oracle.classify_workload(w)


CASES = [
    # (request, verdict, consumed)
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n0\r\n\r\n", ALLOW, None),
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\n", ALLOW, None),
    (HEAD + b"Transfer-Encoding: Chunked \r\n\r\na;x=y\r\n0123456789\r\n0\r\nT: 1\r\nU: 2\r\n\r\n", ALLOW, None),
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n\r\nGET / HTTP/1.1\r\n\r\n", ALLOW, -18),
    (HEAD + b"Transfer-Encoding: chunked\r\nContent-Length: 99\r\n\r\n0\r\n\r\n", ALLOW, None),  # CL ignored
    (HEAD + b"Transfer-Encoding: gzip\r\nContent-Length: 2\r\n\r\nab", ALLOW, None),  # not chunked: CL
    (HEAD + b"Transfer-Encoding: gzip, chunked\r\n\r\n", ALLOW, None),  # not "chunked": no body
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\r\nhel", INCOMPLETE, 0),
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\r\nhello\r\n0\r\n", INCOMPLETE, 0),
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n\r\n", PARSE_ERROR, 0),           # no size digits
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\ng\r\n", PARSE_ERROR, 0),          # not hex
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\nhello\r\n0\r\n\r\n", PARSE_ERROR, 0),  # bare LF
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n5\r\nhelloX\r\n0\r\n\r\n", PARSE_ERROR, 0),  # no CRLF after data
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n100000000\r\n", PARSE_ERROR, 0),  # > 2^32 - 1
    (HEAD + b"Transfer-Encoding: chunked\r\n\r\n0\r\nBad\nTrailer\r\n\r\n", PARSE_ERROR, 0),
]


@pytest.mark.parametrize("i", range(len(CASES)))
def test_chunked_contract(oracle, i):
    req, verdict, consumed = CASES[i]
    v, r, c = run(oracle, [req])
    assert v[0] == verdict
    want = len(req) + consumed if consumed is not None and consumed < 0 else (len(req) if consumed is None else consumed)
    assert c[0] == want


def test_chunked_denied_by_headers(oracle):
    req = b"POST /public/abc/7/x HTTP/1.1\r\nTransfer-Encoding: chunked\r\n\r\n3\r\nabc\r\n0\r\n\r\n"
    v, r, c = run(oracle, [req])
    assert v[0] == DENY and c[0] == len(req)
