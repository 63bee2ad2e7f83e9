"""Device framing of connection streams (l7g_frame_streams /
l7g_classify_streams, kernels/frame.hip) on the GPU.

Each protocol's generated requests are grouped by connection and concatenated
into one stream per connection (some cut short), the way a proxy receives
them.  The frame starts are checked against the oracle's sequential walk: the
proxylib op loop (proxylib/proxylib/connection.go:118-174) hands the parser
the stream from the last frame's end, and the next frame starts where the
oracle's PASS / DROP length (`consumed`) ends it -- Kafka's BE int32 size
prefix (vendor/github.com/optiopay/kafka/proto/messages.go:124-165), memcached
text lines + storage data blocks and binary headers
(proxylib/memcached/{text,binary}/parser.go), HTTP heads + bodies, r2d2 lines,
cassandra headers.  For Kafka and memcached the oracle is the only reference.
For HTTP, r2d2 and cassandra the frames must also equal the restatement below
of the device walk's contract (the parsers' framing as csrc/proxylib/shim.cc
scans it: stop at a Transfer-Encoding head, frame malformed heads by their
"\r\n\r\n"), and, for generated well-formed requests, the request
boundaries.  l7g_classify_streams' verdicts, rule ids and consumed lengths for
every frame equal the oracle's on the same frames."""
import numpy as np
import pytest
import torch

from cilium_amd import gen
from cilium_amd._lib import (ALLOW, DENY, INCOMPLETE, PARSE_ERROR, PROTO_CASSANDRA, PROTO_HTTP, PROTO_KAFKA,
                             PROTO_MEMCACHE, PROTO_R2D2)

pytestmark = pytest.mark.gpu


# ---- the framing restatement (shim.cc NextKafka / NextMcBinary / NextMcText / NextLine / NextHttp)
def _space_len(s, i, n):
    c = s[i]
    if c == 0x20 or 0x09 <= c <= 0x0D:
        return 1
    if c < 0xC2 or c > 0xE3 or i + 1 >= n:
        return 0
    c1 = s[i + 1]
    if c == 0xC2:
        return 2 if c1 in (0x85, 0xA0) else 0
    if i + 2 >= n:
        return 0
    c2 = s[i + 2]
    if c == 0xE1:
        return 3 if (c1, c2) == (0x9A, 0x80) else 0
    if c == 0xE2 and c1 == 0x80:
        return 3 if (0x80 <= c2 <= 0x8A or c2 in (0xA8, 0xA9, 0xAF)) else 0
    if c == 0xE2 and c1 == 0x81:
        return 3 if c2 == 0x9F else 0
    if c == 0xE3:
        return 3 if (c1, c2) == (0x80, 0x80) else 0
    return 0


def _fields(s):
    out, i, start, inside, n = [], 0, 0, False, len(s)
    while i < n:
        sp = _space_len(s, i, n)
        if sp:
            if inside:
                out.append(s[start:i])
            inside = False
            i += sp
        else:
            if not inside:
                start, inside = i, True
            i += 1
    if inside:
        out.append(s[start:])
    return out


def _next(d, p, proto, mode):
    n = len(d)
    if proto == PROTO_KAFKA:
        if n - p < 4:
            return 0
        size = int.from_bytes(d[p:p + 4], "big", signed=True)
        return p + 4 + size if 0 < size and size + 4 <= n - p else 0
    if proto == PROTO_CASSANDRA:
        if n - p < 9:
            return 0
        fl = 9 + int.from_bytes(d[p + 5:p + 9], "big")
        return p + fl if fl <= n - p else 0
    if proto == PROTO_MEMCACHE and mode == 2:
        if n - p < 24:
            return 0
        body = int.from_bytes(d[p + 8:p + 12], "big")
        return p + 24 + body if body + 24 <= n - p else 0
    lf = d.find(b"\r\n", p)
    if lf < 0:
        return 0
    if proto == PROTO_R2D2:
        return lf + 2
    if proto == PROTO_MEMCACHE:
        tok = _fields(d[p:lf])
        nxt = lf + 2
        if tok and tok[0] in (b"set", b"add", b"replace", b"append", b"prepend", b"cas"):
            if len(tok) < 5:
                return 0
            t = tok[4]
            digits = t[1:] if t[:1] in (b"+", b"-") else t
            if not digits or not digits.isdigit():
                return 0
            v = int(digits)
            if t[:1] == b"-" and v:
                return 0
            nxt += v + 2
        return nxt if nxt <= n else 0
    # HTTP
    he = d.find(b"\r\n\r\n", p)
    if he < 0:
        return 0
    cl = 0
    ls = lf + 2
    while ls < he:
        le = d.find(b"\r\n", ls)
        colon = d.find(b":", ls)
        if 0 <= colon < le:
            name = d[ls:colon].lower()
            if name == b"transfer-encoding":
                return 0
            if name == b"content-length":
                v = d[colon + 1:].lstrip(b" \t\r\n\v\f")
                neg = v[:1] == b"-"
                v = v[1:] if v[:1] in (b"+", b"-") else v
                k = 0
                while k < len(v) and 48 <= v[k] <= 57:
                    k += 1
                x = int(v[:k]) if k else 0
                cl = (-x) % (1 << 64) if neg else min(x, (1 << 64) - 1)
        ls = le + 2
    nxt = he + 4 + cl
    return nxt if he + 4 <= n and cl <= n - (he + 4) else 0


def _frames(d, proto, mode, max_frames):
    out, p = [], 0
    if proto == PROTO_MEMCACHE and mode == 0 and d:
        mode = 2 if d[0] >= 0x80 else 1
    while p < len(d) and len(out) < max_frames:
        out.append(p)
        q = _next(d, p, proto, mode)
        if q <= p:
            break
        p = q
    return out


def _oracle_walk(ref, conns, streams, conn_of, max_frames):
    """The oracle's sequential framing of each stream: frame k + 1 starts
    where the oracle's PASS / DROP of frame k (handed the stream from frame
    k's start, as OnData hands the parser its unconsumed input) ends it; the
    walk stops at the first frame the oracle does not pass or drop
    (INCOMPLETE: MORE; PARSE_ERROR: the connection is closed) or at
    max_frames.  Returns per stream the frame starts and the last frame's
    verdict.  All streams advance together, one oracle batch per frame index."""
    arena = np.frombuffer(b"".join(streams), np.uint8).copy()
    base = np.cumsum([0] + [len(s) for s in streams[:-1]]).astype(np.int64)
    # one connection per stream: memcached's parser is chosen by the first byte
    # the connection carries and kept for its lifetime
    # (proxylib/memcached/parser.go:186-199), so the later OnData calls see it
    # locked, as the connection's flags would hold it
    nc = len(conns)
    conns = np.concatenate([conns, np.zeros(len(streams), conns.dtype)])
    for s, st in enumerate(streams):
        c = conn_of[s]
        if c < nc:
            conns[nc + s] = conns[c]
            if int(conns[c]["proto"]) == PROTO_MEMCACHE and int(conns[c]["flags"]) & 3 == 0 and st:
                conns[nc + s]["flags"] = (int(conns[c]["flags"]) & ~3) | (2 if st[0] >= 0x80 else 1)
    conn_of = [nc + s if conn_of[s] < nc else conn_of[s] + len(streams) for s in range(len(streams))]
    pos = [0] * len(streams)
    starts = [[] for _ in streams]
    last = [None] * len(streams)
    live = [s for s in range(len(streams)) if len(streams[s]) > 0]
    while live:
        off = np.array([base[s] + pos[s] for s in live], np.uint64)
        ln = np.array([len(streams[s]) - pos[s] for s in live], np.uint32)
        cid = np.array([conn_of[s] for s in live], np.uint32)
        v, _, c = ref.classify(conns, arena, off, ln, cid, 8)
        nxt = []
        for k, s in enumerate(live):
            starts[s].append(pos[s])
            last[s] = int(v[k])
            if int(v[k]) in (ALLOW, DENY) and 0 < int(c[k]) < len(streams[s]) - pos[s] and \
                    len(starts[s]) < max_frames:
                pos[s] += int(c[k])
                nxt.append(s)
        live = nxt
    return starts, last


def _check_against_oracle_walk(got, want, last, proto, stream, max_frames):
    """The device's frames against the oracle's walk.  They agree on every
    frame both have.  The device may propose frames past one the oracle
    rejects (it frames by length and delimiters only; the caller discards
    them, as proxylib closes the connection), and stops early only where a
    length cannot be read ahead of parsing: a chunked HTTP body (the frame is
    handed the rest of the stream; the classifier frames it)."""
    k = min(len(got), len(want))
    assert got[:k] == want[:k], (proto, got[:8], want[:8])
    if len(got) > len(want):
        assert last == PARSE_ERROR, (proto, len(got), len(want), last)
    elif len(got) < len(want):
        assert proto == PROTO_HTTP and b"transfer-encoding" in stream[got[-1]:].lower(), (proto, got[-3:], want[:len(got) + 1])


def _streams(w, rng, cut_every=5):
    """One stream per connection: its requests in order; every cut_every-th
    stream cut short at a random point."""
    reqs = [bytes(w.arena[int(o):int(o) + int(n)]) for o, n in zip(w.offsets, w.lengths)]
    by = {}
    for q, c in zip(reqs, w.conn_ids):
        # a memcached connection carries one wire format (its first byte picks
        # the parser for good): the generator's text and binary requests of one
        # connection go to two streams
        mc = int(c) < len(w.conns) and int(w.conns["proto"][int(c)]) == PROTO_MEMCACHE and len(q) > 0
        by.setdefault((int(c), mc and q[0] >= 0x80), []).append(q)
    conns, streams, bounds = [], [], []
    for k, ((c, _), qs) in enumerate(sorted(by.items())):
        s = b"".join(qs)
        b = list(np.cumsum([0] + [len(q) for q in qs[:-1]]))
        if k % cut_every == 3 and len(s) > 2:
            s = s[:int(rng.integers(1, len(s)))]
        conns.append(c)
        streams.append(s)
        bounds.append(b)
    return conns, streams, bounds


def _run(engine, oracle, w, max_frames=64, extra=(), streams=None, align=1):
    """extra: (connection, stream) pairs appended to the generated streams;
    streams: (connections, streams, request boundaries) instead of the
    generated ones; align: each stream starts at an arena offset that is a
    multiple of it (the device walk's windows then start at stream offset 0)."""
    rng = np.random.default_rng(7)
    engine.update_policy(w.policy)
    engine.set_connections(w.conns)
    conns, streams, bounds = _streams(w, rng) if streams is None else streams
    for c, st in extra:
        conns.append(c)
        streams.append(st)
        bounds.append([0])
    s_off = np.zeros(len(streams), np.uint64)
    parts, at = [], 0
    for k, st in enumerate(streams):
        pad = (-at) % align
        parts.append(b"\0" * pad)
        at += pad
        s_off[k] = at
        parts.append(st)
        at += len(st)
    arena = np.frombuffer(b"".join(parts) + b"\0", np.uint8).copy()
    s_len = np.array([len(s) for s in streams], np.uint32)
    s_conn = np.array(conns, np.uint32)
    n = len(streams)
    dev = torch.device("cuda", 0)
    t = lambda a: torch.from_numpy(a.view(np.int64) if a.dtype == np.uint64 else a.view(np.int32) if a.itemsize == 4 else a).to(dev)  # noqa: E731
    d_arena, d_off, d_len, d_conn = t(arena), t(s_off), t(s_len), t(s_conn)
    slots = n * max_frames
    f_off = torch.zeros(slots, dtype=torch.int64, device=dev)
    f_len = torch.zeros(slots, dtype=torch.int32, device=dev)
    f_conn = torch.zeros(slots, dtype=torch.int32, device=dev)
    nfr = torch.zeros(n, dtype=torch.int32, device=dev)
    v = torch.zeros(slots, dtype=torch.uint8, device=dev)
    r = torch.zeros(slots, dtype=torch.int32, device=dev)
    c = torch.zeros(slots, dtype=torch.int32, device=dev)
    engine.classify_streams_device(d_arena.data_ptr(), arena.nbytes, d_off.data_ptr(), d_len.data_ptr(),
                                   d_conn.data_ptr(), n, max_frames, f_off.data_ptr(), f_len.data_ptr(),
                                   f_conn.data_ptr(), nfr.data_ptr(), v.data_ptr(), r.data_ptr(), c.data_ptr())
    torch.cuda.synchronize()
    f_off, f_len, f_conn = f_off.cpu().numpy().view(np.uint64), f_len.cpu().numpy().view(np.uint32), \
        f_conn.cpu().numpy().view(np.uint32)
    nfr = nfr.cpu().numpy()
    modes = {i: int(w.conns["flags"][i]) & 3 for i in range(len(w.conns))}
    ref = oracle.Policy(w.policy)
    owalk, olast = _oracle_walk(ref, w.conns, streams, conns, max_frames)
    whole = 0
    sel = []
    for s in range(n):
        got = [int(x) - int(s_off[s]) for x in f_off[s * max_frames:s * max_frames + nfr[s]]]
        if conns[s] >= len(w.conns):  # unknown connection: one slot, the whole stream
            assert got == [0], (s, got)
        else:
            proto = int(w.conns["proto"][conns[s]])
            _check_against_oracle_walk(got, owalk[s], olast[s], proto, streams[s], max_frames)
            if proto not in (PROTO_KAFKA, PROTO_MEMCACHE):  # the device walk's contract, restated
                want = _frames(streams[s], proto, modes[conns[s]], max_frames)
                assert got == want, (s, proto, got[:8], want[:8])
        assert all(int(x) == len(streams[s]) - g for x, g in zip(f_len[s * max_frames:], got))
        assert (f_conn[s * max_frames:s * max_frames + nfr[s]] == conns[s]).all()
        assert (f_len[s * max_frames + nfr[s]:(s + 1) * max_frames] == 0).all()
        if got == [int(b) for b in bounds[s][:len(got)]]:
            whole += 1
        sel.extend(range(s * max_frames, s * max_frames + nfr[s]))
    sel = np.array(sel)
    ref = ref.classify(w.conns, arena, f_off[sel], f_len[sel], f_conn[sel], 8)
    assert (v.cpu().numpy()[sel] == ref[0]).all()
    assert (r.cpu().numpy()[sel] == ref[1]).all()
    assert (c.cpu().numpy().view(np.uint32)[sel] == ref[2]).all()
    empty = np.setdiff1d(np.arange(slots), sel)
    assert (v.cpu().numpy()[empty] == 4).all()  # empty slots: UNSUPPORTED
    return n, whole, len(sel)


@pytest.mark.parametrize("proto", ["http", "kafka", "memcache", "r2d2", "cassandra"])
def test_frame_streams_match_the_scan_and_the_oracle(engine, oracle, proto):
    w = {"http": lambda: gen.http_workload(2, 3000, nconns=64),
         "kafka": lambda: gen.kafka_workload(3000, nconns=64),
         "memcache": lambda: gen.memcache_workload(3000, nconns=64),
         "r2d2": lambda: gen.r2d2_workload(2000, nconns=32),
         "cassandra": lambda: gen.cassandra_workload(2000, nconns=16)}[proto]()
    n, whole, frames = _run(engine, oracle, w)
    assert frames > n * 2  # several frames per stream
    if proto in ("http", "kafka"):  # well-formed generated requests: the frames are the requests
        assert whole >= n * 3 // 4, (whole, n)


@pytest.mark.parametrize("proto", ["http", "kafka"])
def test_frame_streams_max_frames(engine, oracle, proto):
    """More frames than slots: the first max_frames are emitted (the last one
    handed the rest of its stream), as the restatement stops there too."""
    w = {"http": lambda: gen.http_workload(2, 2000, nconns=32),
         "kafka": lambda: gen.kafka_workload(2000, nconns=32)}[proto]()
    n, whole, frames = _run(engine, oracle, w, max_frames=4)
    assert frames == 4 * n and whole == n


def test_frame_streams_edges(engine, oracle):
    """Empty streams (no frame), a stream on an unknown connection (one slot,
    answered as the classifier answers an unknown connection), a stream shorter
    than a Kafka size prefix and one whose size prefix overruns it (one frame
    each, handed the whole stream), next to ordinary streams; and no streams."""
    w = gen.kafka_workload(500, nconns=16)
    unknown = len(w.conns) + 5
    extra = [(0, b""), (1, b"\x00\x00\x00"), (2, b"\x00\x00\x10\x00" + b"x" * 40), (unknown, b"GET / HTTP/1.1\r\n\r\n"),
             (unknown, b""), (3, b"")]
    n, whole, frames = _run(engine, oracle, w, max_frames=8, extra=extra)
    assert frames >= n - 3
    z = torch.zeros(1, dtype=torch.int64, device="cuda")
    engine.classify_streams_device(z.data_ptr(), 0, z.data_ptr(), z.data_ptr(), z.data_ptr(), 0, 8, z.data_ptr(),
                                   z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr(), z.data_ptr())
    torch.cuda.synchronize()


def _http_body_requests(n, seed):
    """Requests whose framing needs the head's content-length / transfer-encoding
    lines: bodies by Content-Length (any case, signs, spaces, overflow), TE
    lines, and long pad headers before and after them so that their line
    starts fall anywhere in the wave framer's 1 KiB windows, window edges
    included."""
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        pad1 = b"a" * int(rng.integers(0, 2400))
        pad2 = b"b" * int(rng.integers(0, 1200))
        body = b"x" * int(rng.integers(0, 300))
        k = int(rng.integers(0, 9))
        name = [b"Content-Length", b"content-length", b"CONTENT-LENGTH", b"Content-Lengthx", b"Content-Length "][
            int(rng.integers(0, 5))]
        val = [b"%d" % len(body), b" %d" % len(body), b"+%d" % len(body), b"-1", b"99999999999999999999999",
               b"\t%d" % len(body), b"%dzz" % len(body), b""][int(rng.integers(0, 8))]
        hdrs = [b"Host: h%d" % i, b"X-Pad: " + pad1]
        if k < 6:
            hdrs.insert(int(rng.integers(0, len(hdrs) + 1)), name + b":" + val)
        if k == 6:
            hdrs.insert(int(rng.integers(0, len(hdrs) + 1)), [b"Transfer-Encoding: chunked", b"transfer-encoding:x",
                                                              b"Transfer-Encodingx: 1"][int(rng.integers(0, 3))])
        if k == 7:  # two content-length lines: the last one counts
            hdrs += [b"Content-Length: 3", b"X-B: " + pad2, b"Content-Length: %d" % len(body)]
        out.append(b"POST /p HTTP/1.1\r\n" + b"\r\n".join(hdrs) + b"\r\n\r\n" + body)
    return out


def test_frame_streams_http_heads_and_bodies(engine, oracle):
    """The wave-per-stream HTTP framer on heads whose content-length and
    transfer-encoding lines decide the frames, the adversarial requests and the
    chunked ones, against the scan restatement and the oracle's verdicts."""
    reqs = _http_body_requests(1500, 21) + gen.http_adversarial(800, 22) + gen.http_chunked(300, 23)
    rng = np.random.default_rng(24)
    reqs = [reqs[i] for i in rng.permutation(len(reqs))]
    arena, offs, lens = gen.pack(reqs)
    base = gen.http_workload(2, 10, nconns=48)
    w = gen.Workload("http-bodies", arena, offs, lens, rng.integers(0, 48, len(reqs)).astype(np.uint32), base.conns,
                     base.policy, {})
    n, whole, frames = _run(engine, oracle, w, max_frames=96)
    assert frames > n * 3


def _edge_requests():
    """HTTP heads whose Content-Length or Transfer-Encoding line starts at
    exactly stream offset 990-995 or 1966-1971: the first bytes past what the
    wave framer's first and second 1 KiB windows vouch for (a window vouches
    for its first 992 bytes; the next starts 976 bytes on).  Each is followed
    by a second request, so a missed length line frames the body as a request."""
    out = []
    line1 = b"POST /p HTTP/1.1\r\n"
    for at in list(range(988, 998)) + list(range(1964, 1974)):
        for hdr in (b"Content-Length: 7", b"content-length:7", b"Transfer-Encoding: chunked"):
            pad = at - len(line1) - len(b"X-Pad: ") - 2
            head = line1 + b"X-Pad: " + b"a" * pad + b"\r\n" + hdr + b"\r\nHost: h\r\n\r\n"
            assert head.index(hdr) == at
            body = b"7\r\nabcdefg\r\n0\r\n\r\n" if hdr.startswith(b"Transfer") else b"GET / H"
            out.append(head + body + b"GET /public/x HTTP/1.1\r\nHost: h\r\n\r\n")
    return out


def test_frame_streams_http_length_line_at_window_edges(engine, oracle):
    """a length line starting at byte 992 / 993 of a window
    was missed.  Every stream starts 16-byte aligned, so its first window
    starts at stream offset 0 and the lines fall on the window edges exactly."""
    reqs = _edge_requests()
    base = gen.http_workload(2, 10, nconns=4)
    conns = [k % 4 for k in range(len(reqs))]
    streams = (conns, list(reqs), [[0] for _ in reqs])
    n, whole, frames = _run(engine, oracle, base, max_frames=4, streams=streams, align=16)
    assert frames >= 2 * n - sum(1 for r in reqs if b"Transfer" in r)
