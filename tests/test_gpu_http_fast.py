"""The latency path's well-formed-head shortcut (http_classify.hip:lat_fast)
against the oracle, bit-exact.

Calls of at most 64 requests run one request per wave; a head that meets
lat_fast's conditions is answered from its closed form, anything else by the
line-parallel framer (lat_request).  These requests sit on both sides of every
condition: HT / SP / DEL / bare CR / bare LF / obs-text in each part of the
head, OWS around slot values (leading, trailing, HT, values of OWS only),
repeated Host and custom headers, names of 15 / 16 bytes and with other
tchars, methods of 16 / 17 bytes, version variants, Content-Length and
Transfer-Encoding lines, header blocks of 61-64 lines, requests cut before
or inside the empty line, and bodies after the head."""
import numpy as np
import pytest

from cilium_amd import gen

from test_gpu_http import wl_from_reqs
from test_gpu_http_latency import _small_calls

pytestmark = pytest.mark.gpu


def near_clean(n, seed):
    rng = np.random.default_rng(seed)
    base = gen.http_requests(n, seed + 1)
    out = []
    for i, r in enumerate(base):
        head, _, rest = r.partition(b"\r\n\r\n")
        lines = head.split(b"\r\n")
        op = int(rng.integers(0, 24))
        if op == 0:  # HT in the target
            lines[0] = lines[0].replace(b" HTTP/", b"\tx HTTP/", 1)
        elif op == 1:  # double SP after the method
            lines[0] = lines[0].replace(b" ", b"  ", 1)
        elif op == 2:  # version variants
            lines[0] = lines[0][:-8] + [b"HTTP/1.0", b"HTTP/2.0", b"http/1.1", b"HTTP/1.", b"HTTP/1.11", b"HTTP/x.1"][int(rng.integers(0, 6))]
        elif op == 3:  # OWS around a slot value (Host / X-Token)
            k = int(rng.integers(1, len(lines)))
            name, _, val = lines[k].partition(b":")
            pre = [b"", b" ", b"\t", b"  \t"][int(rng.integers(0, 4))]
            post = [b"", b" ", b"\t", b" \t ", b"\t\t"][int(rng.integers(0, 5))]
            lines[k] = name + b":" + pre + val.strip(b" ") + post
        elif op == 4:  # value of OWS only / empty value
            k = int(rng.integers(1, len(lines)))
            lines[k] = lines[k].partition(b":")[0] + [b":", b": ", b":\t \t"][int(rng.integers(0, 3))]
        elif op == 5:  # repeated Host (first one counts)
            lines.insert(int(rng.integers(1, len(lines) + 1)), b"Host: svc-%d.other" % int(rng.integers(0, 64)))
        elif op == 6:  # repeated X-Token
            lines.insert(int(rng.integers(1, len(lines) + 1)), b"x-token: %d" % int(rng.integers(0, 10 ** 6)))
        elif op == 7:  # names of 15 / 16 bytes, names with other tchars
            lines.insert(1, [b"X-Abcdefghijklm: 1", b"X-Abcdefghijklmn: 1", b"X_Token: 5", b"X.Y: 2", b"Host_: a"][int(rng.integers(0, 5))])
        elif op == 8:  # method lengths around 16 / other tchars
            m = [b"ABCDEFGHIJKLMNOP", b"ABCDEFGHIJKLMNOPQ", b"G~T", b"GET!", b"get"][int(rng.integers(0, 5))]
            lines[0] = m + b" " + lines[0].partition(b" ")[2]
        elif op == 9:  # Content-Length / Transfer-Encoding
            lines.insert(1, [b"Content-Length: 0", b"Content-Length: 12", b"content-length:  3 ", b"Transfer-Encoding: chunked",
                             b"Content-Length: 1 2"][int(rng.integers(0, 5))])
            rest = b"0\r\n\r\n" if b"chunked" in lines[1] else b"abcdefghijklmnop"
        elif op == 10:  # bare CR / bare LF / DEL / NUL in a value
            k = int(rng.integers(1, len(lines)))
            lines[k] += [b"\rx", b"\nx", b"\x7f", b"\x00", b"\x1b"][int(rng.integers(0, 5))]
        elif op == 11:  # obs-text in the target and in values
            lines[0] = lines[0].replace(b" HTTP/", b"\xc3\xa9\xff HTTP/", 1)
            lines[1] += b"\xe2\x82\xac"
        elif op == 12:  # obs-fold
            lines.insert(2, b" folded")
        elif op == 13:  # empty name / no colon
            lines.insert(1, [b": v", b"NoColon", b"Name : v"][int(rng.integers(0, 3))])
        elif op == 14:  # many lines: the 62-line limit
            lines[1:1] = [b"X-L%d: v" % j for j in range(int(rng.integers(56, 64)))]
        elif op == 15:  # cut before / inside the empty line
            out.append((b"\r\n".join(lines) + [b"", b"\r\n", b"\r\n\r"][int(rng.integers(0, 3))]))
            continue
        elif op == 16:  # leading CRLF / SP
            lines[0] = [b"\r\n", b" "][int(rng.integers(0, 2))] + lines[0]
        elif op == 17:  # DEL / CTL in the method or the target
            lines[0] = lines[0].replace(b"/", [b"/\x7f", b"/\x01", b"/\x09"][int(rng.integers(0, 3))], 1)
        elif op == 18:  # case of slot names
            lines = [ln.replace(b"Host:", b"HOST:").replace(b"X-Token:", b"x-TOKEN:") for ln in lines]
        elif op == 19:  # a body after the head (no Content-Length)
            rest += b"GET /next HTTP/1.1\r\n\r\n"
        out.append(b"\r\n".join(lines) + b"\r\n\r\n" + rest)
    return out


@pytest.mark.parametrize("seed", [11, 12])
def test_fast_path_edges(engine, oracle, seed):
    reqs = near_clean(4000, seed)
    base = gen.http_workload(2, 1)
    rng = np.random.default_rng(seed)
    w = wl_from_reqs(reqs, base.policy, base.conns, rng.integers(0, len(base.conns), len(reqs)))
    _small_calls(engine, oracle, w, seed=seed, nmax=8)


def test_fast_path_cfg1_rules(engine, oracle):
    """cfg1's rule set (one method + path rule: no header slots) on the same heads."""
    reqs = near_clean(2000, 21)
    base = gen.http_workload(1, 1)
    rng = np.random.default_rng(21)
    w = wl_from_reqs(reqs, base.policy, base.conns, rng.integers(0, len(base.conns), len(reqs)))
    _small_calls(engine, oracle, w, seed=21, nmax=8)
