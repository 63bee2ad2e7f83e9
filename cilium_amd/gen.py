"""Deterministic synthetic workloads.

Every generator returns a Workload: one packed payload arena, per-request
(offset, length, connection) arrays, the connection table and the policy set
(cilium.NetworkPolicy JSON).  Seeds are 0x1C1D0000 + config number.

cfg1  1 rule  {Method:"GET", Path:"/public/.*"}                  (HTTP)
cfg2  64 HTTP rules over Method/Path/Host + literal X-Token header  (HTTP, bench)
cfg3  Kafka produce/fetch/metadata stream, ~1k PortRuleKafka rules  (Kafka)
cfg4  10k HTTP rules across 512 identities                          (HTTP)
cfg5  mixed stream 50 % HTTP / 30 % Kafka / 20 % memcached (text + binary)
      memcached part: text and binary commands against the mc rules below
"""
import struct
import zlib
from dataclasses import dataclass, field

import numpy as np

from . import api
from ._lib import PROTO_CASSANDRA, PROTO_HTTP, PROTO_KAFKA, PROTO_MEMCACHE, PROTO_R2D2
from .engine import CONN_DTYPE

SEED_BASE = 0x1C1D0000


@dataclass
class Workload:
    name: str
    arena: np.ndarray            # uint8
    offsets: np.ndarray          # uint64
    lengths: np.ndarray          # uint32
    conn_ids: np.ndarray         # uint32
    conns: np.ndarray            # CONN_DTYPE
    policy: dict                 # policy set JSON (dict)
    meta: dict = field(default_factory=dict)

    @property
    def n(self):
        return len(self.offsets)

    def subset(self, idx):
        idx = np.asarray(idx)
        return Workload(self.name + "[sub]", self.arena, self.offsets[idx], self.lengths[idx],
                        self.conn_ids[idx], self.conns, self.policy, self.meta)

    def algorithmic_bytes(self):
        """B_i = len_i + 16 (offset u64 + len u32 + meta u32) + 9 (verdict u8 + rule i32 + consumed u32).

        memcached requests count only the bytes the parser must inspect (the
        command line, or the 24-byte header + extras + key): the data block of a
        storage command is framed by its length and never read
        (text/parser.go:186-198, binary/parser.go:86-105).  Generators that
        know this set meta["payload_bytes"]."""
        payload = self.meta.get("payload_bytes")
        if payload is None:
            payload = int(self.lengths.astype(np.int64).sum())
        return int(payload) + 25 * self.n


def pack(reqs):
    lens = np.fromiter((len(r) for r in reqs), dtype=np.uint32, count=len(reqs))
    offs = np.zeros(len(reqs), dtype=np.uint64)
    if len(reqs) > 1:
        offs[1:] = np.cumsum(lens[:-1], dtype=np.uint64)
    arena = np.frombuffer(b"".join(reqs), dtype=np.uint8).copy()
    return arena, offs, lens


def make_conns(n, policy, port, ingress, proto, src_ids, dst_id=7):
    c = np.zeros(n, CONN_DTYPE)
    c["policy"] = policy
    c["port"] = port
    c["ingress"] = 1 if ingress else 0
    c["proto"] = proto
    c["src_id"] = src_ids
    c["dst_id"] = dst_id
    return c


# ------------------------------------------------------------------ HTTP
_ALNUM = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789", dtype=np.uint8)
_PATHCH = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz0123456789/_-", dtype=np.uint8)
_LOWER = np.frombuffer(b"abcdefghijklmnopqrstuvwxyz", dtype=np.uint8)
_PAD = bytes((b"abcdefghijklmnopqrstuvwxyzABCDEFGHIJKLMNOPQRSTUVWXYZ0123456789" * 40)[:2100])
_METHODS = [b"GET", b"POST", b"PUT", b"DELETE", b"PATCH"]


def _rand_str(rng, alphabet, lo, hi, n):
    lens = rng.integers(lo, hi + 1, size=n)
    buf = alphabet[rng.integers(0, len(alphabet), size=int(lens.sum()))].tobytes()
    out, p = [], 0
    for L in lens:
        out.append(buf[p:p + L])
        p += L
    return out


def http_requests(n, seed, with_token=True):
    """The §8(d) HTTP template; total length uniform in [256, 2048]."""
    rng = np.random.default_rng(seed)
    meth = rng.choice(5, p=[0.6, 0.2, 0.1, 0.05, 0.05], size=n)
    kind = rng.choice(3, p=[0.5, 0.3, 0.2], size=n)
    words = _rand_str(rng, _LOWER, 3, 8, n)
    # paths and hosts are correlated the way a real client population targets
    # services, so the cfg2/cfg4 rules (which pin service, version and host
    # together) match a realistic share of requests instead of ~0
    nums = np.where(rng.random(n) < 0.6, 2 * rng.integers(0, 32, size=n) + 1, rng.integers(0, 100, size=n))
    tails = _rand_str(rng, _PATHCH, 0, 40, n)
    svc = rng.integers(0, 64, size=n)
    ver = np.where(rng.random(n) < 0.8, svc % 3 + 1, rng.integers(1, 4, size=n))
    target = np.where(kind == 0, nums % 64, svc)
    host = np.where(rng.random(n) < 0.8, target, rng.integers(0, 64, size=n))
    tok_kind = rng.choice(4, p=[0.5, 0.25, 0.24, 0.01], size=n)  # digits / alnum / absent / literal
    tok_digits = _rand_str(rng, np.frombuffer(b"0123456789", np.uint8), 8, 16, n)
    tok_alnum = _rand_str(rng, _ALNUM, 8, 16, n)
    total = rng.integers(256, 2049, size=n)
    padoff = rng.integers(0, 40, size=n)
    reqs = []
    for i in range(n):
        k = kind[i]
        if k == 0:
            path = b"/public/%s/%d/%s" % (words[i], nums[i], tails[i])
        elif k == 1:
            path = b"/private/" + tails[i]
        else:
            path = b"/api/v%d/svc%d/%s" % (ver[i], svc[i], tails[i])
        head = b"%s %s HTTP/1.1\r\nHost: svc-%d.ns.svc.cluster.local\r\nUser-Agent: l7bench/1\r\nAccept: */*\r\n" % (
            _METHODS[meth[i]], path, host[i])
        if with_token:
            t = tok_kind[i]
            if t == 0:
                head += b"X-Token: " + tok_digits[i] + b"\r\n"
            elif t == 1:
                head += b"X-Token: " + tok_alnum[i] + b"\r\n"
            elif t == 3:
                head += b"X-Token: [0-9]+\r\n"
        padlen = max(0, int(total[i]) - len(head) - 11)
        reqs.append(head + b"X-Pad: " + _PAD[padoff[i]:padoff[i] + padlen] + b"\r\n\r\n")
    return reqs


def cfg1_policy():
    rules = api.http_rules_from_api([api.PortRuleHTTP(method="GET", path="/public/.*")])
    return api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(80, [api.port_rule(http=rules)])]))


def cfg2_rules(k0=0, count=64):
    out = []
    for k in range(k0, k0 + count):
        method = ["GET", "POST", "PUT|PATCH", "(GET|HEAD)"][k % 4]
        path = f"/api/v{k % 3 + 1}/svc{k % 64}/.*" if k % 2 == 0 else f"/public/[a-z]+/{k % 100}/.*"
        host = f"svc-{k % 64}\\..*"
        headers = ["X-Token: [0-9]+"] if k % 4 == 3 else []
        out.append(api.PortRuleHTTP(method=method, path=path, host=host, headers=headers))
    return out


def cfg2_policy():
    rules = api.http_rules_from_api(cfg2_rules())
    return api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(80, [api.port_rule(http=rules)])]))


def http_workload(cfg, n, nconns=1024, seed=None):
    seed = SEED_BASE + cfg if seed is None else seed
    reqs = http_requests(n, seed, with_token=(cfg != 1))
    arena, offs, lens = pack(reqs)
    rng = np.random.default_rng(seed + 1)
    conn_ids = rng.integers(0, nconns, size=n).astype(np.uint32)
    conns = make_conns(nconns, 0, 80, True, PROTO_HTTP, 1000 + np.arange(nconns))
    pol = cfg1_policy() if cfg == 1 else cfg2_policy()
    return Workload(f"cfg{cfg}", arena, offs, lens, conn_ids, conns, pol)


def cfg4_workload(n, nids=512, rules_total=10000, seed=None, unknown_frac=0.02):
    """10k HTTP rules across 512 identities (ids 256..767), ~20 rules each as
    separate PortNetworkPolicyRule groups; requests from connections whose
    source identity is uniform over the 512 (+2% unknown => deny)."""
    seed = SEED_BASE + 4 if seed is None else seed
    rng = np.random.default_rng(seed)
    per, extra = divmod(rules_total, nids)  # the first `extra` identities get one more rule
    groups = []
    for g in range(nids):
        ks = rng.integers(0, 4096, size=per + (1 if g < extra else 0))
        rules = [cfg2_rules(int(k), 1)[0] for k in ks]
        groups.append(api.port_rule(remote_policies=[256 + g], http=api.http_rules_from_api(rules)))
    pol = api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(80, groups)]))
    reqs = http_requests(n, seed + 7)
    arena, offs, lens = pack(reqs)
    nconns = nids * 4 + 64
    ids = np.concatenate([256 + np.repeat(np.arange(nids), 4), 5000 + np.arange(64)])
    conns = make_conns(nconns, 0, 80, True, PROTO_HTTP, ids)
    known = rng.random(n) >= unknown_frac
    conn_ids = np.where(known, rng.integers(0, nids * 4, size=n), nids * 4 + rng.integers(0, 64, size=n))
    return Workload("cfg4", arena, offs, lens, conn_ids.astype(np.uint32), conns, pol)


# ------------------------------------------------------------------ adversarial HTTP
_SPECIALS = [b" ", b"\r", b"\n", b"\t", b":", b"\x00", b"\x7f", b"\xff", b"\xc3\xa9", b"\r\n", b"\r\n\r\n",
             b"Content-Length: 5\r\n", b"Transfer-Encoding: chunked\r\n", b"Host: evil\r\n", b" x", b"HTTP/1.1"]


def http_adversarial(n, seed):
    """Valid template requests with random mutations (substitute / insert /
    delete / truncate / duplicate headers) to exercise framing precedence."""
    base = http_requests(n, seed)
    rng = np.random.default_rng(seed + 99)
    out = []
    for i, r in enumerate(base):
        r = bytearray(r[: int(rng.integers(64, 400))] + b"X-Pad: q\r\n\r\n") if rng.random() < 0.5 else bytearray(r)
        for _ in range(int(rng.integers(0, 4))):
            op = rng.integers(0, 5)
            p = int(rng.integers(0, max(1, len(r))))
            if op == 0:
                s = _SPECIALS[int(rng.integers(0, len(_SPECIALS)))]
                r[p:p + len(s)] = s
            elif op == 1:
                r[p:p] = _SPECIALS[int(rng.integers(0, len(_SPECIALS)))]
            elif op == 2:
                del r[p:p + int(rng.integers(1, 4))]
            elif op == 3:
                r = r[:p]
            else:
                r = r + b"GET / HTTP/1.1\r\n\r\n"
        if rng.random() < 0.1 and r.endswith(b"\r\n\r\n"):
            r = r[:-2] + b"Content-Length: %d\r\n\r\n" % int(rng.integers(0, 20)) + bytes(int(rng.integers(0, 25)))
        out.append(bytes(r))
    return out


def http_chunked(n, seed):
    """Requests with Transfer-Encoding (DESIGN.md §4 chunked-body contract):
    valid chunked bodies (0-5 chunks, hex sizes in either case, chunk
    extensions, trailers), TE values that are and are not "chunked", TE with
    Content-Length, then truncations and byte edits anywhere in the framing."""
    rng = np.random.default_rng(seed)
    D = _Draws(rng, 64 * n + 1024)
    heads = http_requests(n, seed + 1)
    te_vals = [b"chunked", b"Chunked", b"CHUNKED", b"chunked  ", b"chunked\t", b"gzip", b"gzip, chunked",
               b"chunkedx", b"chun ked", b"identity"]
    out = []
    for i in range(n):
        h = heads[i]
        h = h[:h.index(b"X-Pad:")]  # request line + Host / UA / Accept / X-Token
        te = te_vals[D.int(0, len(te_vals))] if D.uniform() < 0.5 else b"chunked"
        h += b"Transfer-Encoding: " + te + b"\r\n"
        if D.uniform() < 0.15:
            h += b"Content-Length: %d\r\n" % D.int(0, 20)
        if D.uniform() < 0.05:
            h += b"Transfer-Encoding: " + te_vals[D.int(0, len(te_vals))] + b"\r\n"
        body = b""
        for _ in range(D.int(0, 6)):
            size = D.int(1, 300)
            hx = (b"%x" if D.uniform() < 0.5 else b"%X") % size
            if D.uniform() < 0.1:
                hx = b"0" * D.int(1, 3) + hx
            ext = b";name=val" if D.uniform() < 0.2 else b""
            body += hx + ext + b"\r\n" + D.bytes(size) + b"\r\n"
        body += b"0" + (b";last" if D.uniform() < 0.1 else b"") + b"\r\n"
        if D.uniform() < 0.3:
            body += b"X-Trailer: t%d\r\n" % i
        body += b"\r\n"
        r = bytearray(h + b"\r\n" + body)
        if D.uniform() < 0.2:
            r += b"GET / HTTP/1.1\r\n\r\n"  # a pipelined next request
        op = D.int(0, 10)
        if op == 0:
            r = r[:D.int(len(h), len(r) + 1)]
        elif op == 1 and len(r) > len(h) + 2:
            p = D.int(len(h) + 2, len(r))
            r[p] = [0x0D, 0x0A, 0x3B, 0x47, 0x20, 0x00, 0x30][D.int(0, 7)]
        elif op == 2:
            r = r.replace(b"\r\n0\r\n", b"\r\nfffffffff\r\n", 1)
        out.append(bytes(r))
    return out


# ------------------------------------------------------------------ Kafka wire encoder
# Restates the optiopay/kafka proto encoders the reference's decoders expect
# (vendor/github.com/optiopay/kafka/proto/messages.go: *Req.Bytes).

def k_str(s):
    if s is None:
        return struct.pack(">h", -1)
    b = s.encode() if isinstance(s, str) else s
    return struct.pack(">h", len(b)) + b


def k_bytes(b):
    if b is None:
        return struct.pack(">i", -1)
    return struct.pack(">i", len(b)) + b


def k_message(value, key=None, version=0, attributes=0, timestamp=0, bad_crc=False):
    """One message-set entry: offset i64, size i32, crc u32, magic, attributes,
    [timestamp i64 when the *API version* >= 1 (readMessageSet quirk)], key, value."""
    body = struct.pack(">bb", 1 if version >= 1 else 0, attributes)
    if version >= 1:
        body += struct.pack(">q", timestamp)
    body += k_bytes(key) + k_bytes(value)
    crc = zlib.crc32(body) & 0xFFFFFFFF
    if bad_crc:
        crc ^= 0x5A5A5A5A
    msg = struct.pack(">I", crc) + body
    return struct.pack(">qi", 0, len(msg)) + msg


def snappy_block(data, copies=True):
    """A plain snappy block (varint length + literal / copy tags), greedy over
    4-byte matches; copies=False emits literals only.  For test streams."""
    out = bytearray()
    n = len(data)
    v = n
    while True:
        b = v & 0x7F
        v >>= 7
        out.append(b | (0x80 if v else 0))
        if not v:
            break

    def literal(lo, hi):
        while lo < hi:
            k = min(hi - lo, 1 << 16)
            if k <= 60:
                out.append((k - 1) << 2)
            elif k <= 256:
                out.extend(bytes([60 << 2, k - 1]))
            else:
                out.extend(bytes([61 << 2]) + struct.pack("<H", k - 1))
            out.extend(data[lo:lo + k])
            lo += k

    last, i, table = 0, 0, {}
    while copies and i + 4 <= n:
        key = bytes(data[i:i + 4])
        j = table.get(key)
        table[key] = i
        if j is not None and 0 < i - j < 65536:
            m = 4
            while i + m < n and m < 64 and data[j + m] == data[i + m]:
                m += 1
            literal(last, i)
            out += bytes([((m - 1) << 2) | 2]) + struct.pack("<H", i - j)
            i += m
            last = i
        else:
            i += 1
    literal(last, n)
    return bytes(out)


def snappy_xerial(data, chunk=4096, copies=True):
    """snappy-java (xerial) framing: magic, version 1, compat 1, then
    (BE32 length, snappy block) per chunk."""
    out = b"\x82SNAPPY\x00" + struct.pack(">ii", 1, 1)
    for o in range(0, len(data), chunk):
        blk = snappy_block(data[o:o + chunk], copies)
        out += struct.pack(">i", len(blk)) + blk
    return out


def k_compressed(inner, codec, version=0, timestamp=0, xerial=False, gzip_kwargs=None):
    """A message whose value is the message set `inner` (bytes) compressed:
    codec 1 = gzip, 2 = snappy (messages.go:460-489)."""
    if codec == 1:
        import gzip as _gz
        value = _gz.compress(inner, **(gzip_kwargs or {}))
    else:
        value = snappy_xerial(inner) if xerial else snappy_block(inner)
    return k_message(value, key=None, version=version, attributes=codec, timestamp=timestamp)


def k_request(kind, version, corr, client, body):
    payload = struct.pack(">hhi", kind, version, corr) + k_str(client) + body
    return struct.pack(">i", len(payload)) + payload


def k_produce(version, corr, client, topics, acks=-1, timeout=1000, txn=None):
    """topics: list of (name, [(partition, [message bytes...]), ...])"""
    b = b""
    if version >= 3:
        b += k_str(txn)
    b += struct.pack(">hi", acks, timeout) + struct.pack(">i", len(topics))
    for name, parts in topics:
        b += k_str(name) + struct.pack(">i", len(parts))
        for pid, msgs in parts:
            ms = b"".join(msgs)
            b += struct.pack(">ii", pid, len(ms)) + ms
    return k_request(0, version, corr, client, b)


def k_fetch(version, corr, client, topics):
    """topics: list of (name, [partition ids])"""
    b = struct.pack(">iii", -1, 100, 1)
    if version >= 3:
        b += struct.pack(">i", 1 << 20)
    if version >= 4:
        b += struct.pack(">b", 0)
    b += struct.pack(">i", len(topics))
    for name, parts in topics:
        b += k_str(name) + struct.pack(">i", len(parts))
        for pid in parts:
            b += struct.pack(">iq", pid, 0)
            if version >= 5:
                b += struct.pack(">q", 0)
            b += struct.pack(">i", 1 << 16)
    return k_request(1, version, corr, client, b)


def k_metadata(version, corr, client, topics):
    b = struct.pack(">i", -1) if topics is None else struct.pack(">i", len(topics)) + b"".join(k_str(t) for t in topics)
    if version >= 4:
        b += b"\x01"
    return k_request(3, version, corr, client, b)


def k_offset(version, corr, client, topics):
    """ListOffsets (kind 2): topics: list of (name, [partition ids])"""
    b = struct.pack(">i", -1)
    if version >= 2:
        b += b"\x00"
    b += struct.pack(">i", len(topics))
    for name, parts in topics:
        b += k_str(name) + struct.pack(">i", len(parts))
        for pid in parts:
            b += struct.pack(">iq", pid, -1)
            if version == 0:
                b += struct.pack(">i", 1)
    return k_request(2, version, corr, client, b)


def k_offset_commit(version, corr, client, group, topics):
    """OffsetCommit (kind 8): topics: list of (name, [partition ids])"""
    b = k_str(group)
    if version >= 1:
        b += struct.pack(">i", 3) + k_str("member-1")
    if version >= 2:
        b += struct.pack(">q", 60000)
    b += struct.pack(">i", len(topics))
    for name, parts in topics:
        b += k_str(name) + struct.pack(">i", len(parts))
        for pid in parts:
            b += struct.pack(">iq", pid, 42)
            if version == 1:
                b += struct.pack(">q", 1234)
            b += k_str("meta")
    return k_request(8, version, corr, client, b)


def k_offset_fetch(version, corr, client, group, topics):
    """OffsetFetch (kind 9): topics None (null array) or list of (name, [partition ids])"""
    b = k_str(group)
    if topics is None:
        b += struct.pack(">i", -1)
    else:
        b += struct.pack(">i", len(topics))
        for name, parts in topics:
            b += k_str(name) + struct.pack(">i", len(parts)) + b"".join(struct.pack(">i", p) for p in parts)
    return k_request(9, version, corr, client, b)


def k_consumer_metadata(version, corr, client, group):
    b = k_str(group)
    if version >= 1:
        b += b"\x00"
    return k_request(10, version, corr, client, b)


def kafka_all_kinds(n, seed):
    """Every kind the reference decodes (0, 1, 2, 3, 8, 9, 10) plus untyped
    ones, at every version the decoders distinguish, with 0-5 topics of
    1-3 partitions (parity coverage for the decode program of each kind)."""
    rng = np.random.default_rng(seed)
    topics = kafka_topics()
    D = _Draws(rng, 64 * n + 1024)
    out = []

    def tps(with_parts=True):
        k = D.int(0, 6)
        return [(topics[D.int(0, 1000)] if D.uniform() < 0.9 else "", [D.int(0, 8) for _ in range(D.int(1, 4))])
                for _ in range(k)]

    for i in range(n):
        client = f"client-{D.int(0, 16):02d}" if D.uniform() < 0.95 else ""
        k = D.int(0, 9)
        if k == 0:
            v = D.int(0, 4)
            t = [(name, [(p, [k_message(D.bytes(D.int(0, 90)), version=v) for _ in range(D.int(0, 3))])
                         for p in parts]) for name, parts in tps()]
            out.append(k_produce(v, i, client, t, txn="tx" if v >= 3 and D.uniform() < 0.5 else None))
        elif k == 1:
            out.append(k_fetch(D.int(0, 6), i, client, tps()))
        elif k == 2:
            out.append(k_offset(D.int(0, 3), i, client, tps()))
        elif k == 3:
            out.append(k_metadata(D.int(0, 6), i, client, None if D.uniform() < 0.2 else [n for n, _ in tps()]))
        elif k == 4:
            out.append(k_offset_commit(D.int(0, 4), i, client, "grp", tps()))
        elif k == 5:
            out.append(k_offset_fetch(D.int(0, 4), i, client, "grp", None if D.uniform() < 0.2 else tps()))
        elif k == 6:
            out.append(k_consumer_metadata(D.int(0, 2), i, client, "grp"))
        elif k == 7:
            out.append(k_request(int(rng.choice([4, 5, 6, 7, 11, 12, 18, 19, 36])), D.int(0, 3), i, client, b"\x00" * D.int(0, 12)))
        else:  # truncated or size-edited frames of the above kinds
            r = bytearray(k_offset_commit(D.int(0, 4), i, client, "grp", tps()) if D.uniform() < 0.5
                          else k_offset(D.int(0, 3), i, client, tps()))
            cut = D.int(12, len(r) + 1)
            r = r[:cut]
            if D.uniform() < 0.5:
                r[0:4] = struct.pack(">i", len(r) - 4)
            out.append(bytes(r))
    return out


def kafka_topics():
    return [f"topic-{i:04d}" for i in range(1000)]


def cfg3_rules():
    topics = kafka_topics()
    rules = [api.PortRuleKafka(role="produce", topic=topics[i]) for i in range(500)]
    rules += [api.PortRuleKafka(api_key="fetch", topic=topics[500 + j], client_id=f"client-{j % 16:02d}")
              for j in range(500)]
    rules += [api.PortRuleKafka(api_key="metadata"), api.PortRuleKafka(api_key="apiversions")]
    return rules


def cfg3_policy():
    return api.policy_set(api.network_policy("10.0.0.1", 3, ingress=[(9092, [api.port_rule(kafka=cfg3_rules())])]))


class _Draws:
    """Scalar draws from pre-generated uniforms (numpy per-call overhead
    dominated the per-request generators)."""

    def __init__(self, rng, n):
        self.u = rng.random(n).tolist()
        self.k = 0
        self.pool = rng.integers(0, 256, size=1 << 22, dtype=np.uint8).tobytes()
        self.pk = 0

    def uniform(self):
        if self.k >= len(self.u):
            self.k = 0
        v = self.u[self.k]
        self.k += 1
        return v

    def int(self, lo, hi):
        """uniform integer in [lo, hi)"""
        return lo + int(self.uniform() * (hi - lo))

    def bytes(self, n):
        if self.pk + n > len(self.pool):
            self.pk = 0
        b = self.pool[self.pk:self.pk + n]
        self.pk += n + 1
        return b


def kafka_requests(n, seed):
    rng = np.random.default_rng(seed)
    topics = kafka_topics()
    kind = rng.choice(3, p=[0.5, 0.4, 0.1], size=n)
    D = _Draws(rng, 64 * n + 1024)
    out = []

    def pick_topic():
        if D.uniform() < 0.9:
            return topics[D.int(0, 1000)]
        return f"other-{D.int(0, 1000):04d}"

    for i in range(n):
        client = f"client-{D.int(0, 16):02d}"
        if kind[i] == 0:
            v = D.int(0, 3)
            tps = []
            for _ in range(D.int(1, 4)):
                msgs = [k_message(D.bytes(D.int(64, 513)), key=None if D.uniform() < 0.5 else b"k%d" % i, version=v)
                        for _ in range(D.int(1, 5))]
                tps.append((pick_topic(), [(0, msgs)]))
            out.append(k_produce(v, i, client, tps))
        elif kind[i] == 1:
            v = D.int(0, 6)
            tps = [(pick_topic(), [D.int(0, 8)]) for _ in range(D.int(1, 5))]
            out.append(k_fetch(v, i, client, tps))
        else:
            sub = D.int(0, 3)
            if sub == 0:
                tl = None if D.uniform() < 0.3 else [pick_topic() for _ in range(D.int(0, 4))]
                out.append(k_metadata(D.int(0, 6), i, client, tl))
            elif sub == 1:
                out.append(k_request(18, 0, i, client, b""))  # ApiVersions
            else:
                out.append(k_request(12, 0, i, client, k_str("group") + struct.pack(">i", 1) + k_str("m")))  # Heartbeat
    return out


def kafka_adversarial(n, seed):
    """Mutated Kafka frames: bad CRCs, truncation, size/array-length edits,
    compressed sets, unknown kinds, negative string lengths."""
    rng = np.random.default_rng(seed)
    base = kafka_requests(n, seed + 5)
    out = []
    for r in base:
        r = bytearray(r)
        op = int(rng.integers(0, 10))
        if op == 0 and len(r) > 40:  # flip a byte somewhere in the body
            p = int(rng.integers(12, len(r)))
            r[p] ^= int(rng.integers(1, 256))
        elif op == 1:  # truncate the frame but keep the declared size
            r = r[: int(rng.integers(0, len(r)))]
        elif op == 2:  # declared size smaller than the body (trailing bytes ignored / short reads)
            newsize = int(rng.integers(0, max(1, len(r) - 4)))
            r[0:4] = struct.pack(">i", newsize)
        elif op == 3:  # negative or huge sizes
            r[0:4] = struct.pack(">i", int(rng.choice([-1, 0, 3, 7, 6553500, 6553497])))
        elif op == 4:  # unknown / odd kinds
            r[4:6] = struct.pack(">h", int(rng.choice([-1, 7, 19, 33, 64, 1000, 10])))
        elif op == 5:  # version edits
            r[6:8] = struct.pack(">h", int(rng.integers(-2, 8)))
        elif op == 6:  # produce with a corrupt CRC in the middle message / compressed set
            v = int(rng.integers(0, 3))
            msgs = [k_message(b"x" * 70, version=v), k_message(b"y" * 70, version=v, bad_crc=True),
                    k_message(b"z" * 70, version=v)]
            tps = [("topic-0001", [(0, msgs)]), ("topic-0002", [(0, [k_message(b"w" * 80, version=v)])])]
            if rng.random() < 0.3:
                tps = [("topic-0003", [(0, [k_message(b"c" * 90, version=v, attributes=int(rng.integers(1, 4)))])])]
            r = bytearray(k_produce(v, 7, "client-01", tps))
        elif op == 7:  # negative array length
            p = 14 + int.from_bytes(r[12:14], "big", signed=True) if len(r) > 14 else 12
            if 0 < p < len(r) - 4:
                r[p:p + 4] = struct.pack(">i", -int(rng.integers(1, 3)))
        elif op == 8:  # negative string length for the client id
            if len(r) > 14:
                r[12:14] = struct.pack(">h", -int(rng.integers(1, 5)))
        out.append(bytes(r))
    return out


def _gz_member(data, level=6, strategy=0, flags=0, extra=b"", name=b"", comment=b"", hcrc=False, zdict=None):
    """One gzip member built field by field (header flags, raw DEFLATE with a
    chosen strategy / preset history, CRC32 + ISIZE trailer)."""
    h = bytes([0x1F, 0x8B, 8, flags | (0x02 if hcrc else 0)]) + b"\0\0\0\0\0\xff"
    if flags & 0x04:
        h += struct.pack("<H", len(extra)) + extra
    if flags & 0x08:
        h += name + b"\0"
    if flags & 0x10:
        h += comment + b"\0"
    if hcrc:
        h += struct.pack("<H", zlib.crc32(h) & 0xFFFF)
    kw = {"zdict": zdict} if zdict else {}
    c = zlib.compressobj(level, zlib.DEFLATED, -15, 9, strategy, **kw)
    body = c.compress(data) + c.flush()
    return h + body + struct.pack("<II", zlib.crc32(data) & 0xFFFFFFFF, len(data) & 0xFFFFFFFF)


def snappy_far_copy(data, dist):
    """A snappy block of `data` followed by a copy of its first 64 bytes taken
    `dist` (> 65535) back with a 4-byte-offset tag."""
    assert dist >= len(data) and dist >= 65536
    body = data + bytes(dist - len(data))
    v, out = len(body) + 64, bytearray()  # literals of body, then one copy-4 tag of 64 bytes
    while True:
        b, v = v & 0x7F, v >> 7
        out.append(b | (0x80 if v else 0))
        if not v:
            break
    for lo in range(0, len(body), 1 << 16):
        k = min(len(body) - lo, 1 << 16)
        out.extend(bytes([61 << 2]) + struct.pack("<H", k - 1) + body[lo:lo + k])
    out.extend(bytes([(63 << 2) | 3]) + struct.pack("<I", dist))
    return bytes(out)


def kafka_compressed_requests(n, seed):
    """Produce requests whose partitions mix plain and compressed messages:
    gzip (levels 0-9, fixed / huffman-only / RLE strategies, header fields,
    several members), snappy (plain and xerial, long offsets), nesting, and
    corrupted compressed values whose message CRCs are valid, so the decoders
    see the damage."""
    rng = np.random.default_rng(seed)
    topics = ["topic-%04d" % i for i in range(20)]
    out = []

    def payload(k):
        a = [b"abcabcabd ", b"kafka-record-%d;", b"\x00\x01\x02\x03"][int(rng.integers(0, 3))]
        if b"%d" in a:
            s = b"".join(a % int(rng.integers(0, 50)) for _ in range(k // 12 + 1))
        else:
            s = a * (k // len(a) + 1)
        s = bytearray(s[:k])
        for _ in range(int(rng.integers(0, 4))):
            if s:
                s[int(rng.integers(0, len(s)))] = int(rng.integers(0, 256))
        return bytes(s)

    def inner(ver, depth=0):
        msgs = []
        for _ in range(int(rng.integers(1, 4))):
            if depth < 2 and rng.random() < 0.15:
                msgs.append(compressed(inner(ver, depth + 1), ver))
            else:
                msgs.append(k_message(payload(int(rng.integers(0, 600))), version=ver))
        return b"".join(msgs)

    def compressed(data, ver):
        c = int(rng.integers(0, 8))
        if c < 4:
            value = _gz_member(data, level=int(rng.integers(0, 10)),
                               strategy=int(rng.choice([0, 0, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE])),
                               flags=int(rng.choice([0, 0, 0x04, 0x08, 0x1C])), extra=b"xy", name=b"f.bin",
                               comment=b"c", hcrc=bool(rng.random() < 0.2))
            if rng.random() < 0.15:  # a second member
                value += _gz_member(payload(int(rng.integers(0, 50))))
            codec = 1
        else:
            value = snappy_xerial(data, chunk=int(rng.integers(100, 5000))) if c >= 6 else snappy_block(data)
            codec = 2
        if rng.random() < 0.25:  # damage the compressed bytes (the message CRC stays valid)
            value = bytearray(value)
            op = int(rng.integers(0, 3))
            if op == 0 and value:
                i = int(rng.integers(0, len(value)))
                value[i] ^= 1 << int(rng.integers(0, 8))
            elif op == 1 and value:
                del value[int(rng.integers(0, len(value))):]
            else:
                value += bytes(int(rng.integers(1, 12)))
            value = bytes(value)
        return k_message(value, version=ver, attributes=codec)

    for i in range(n):
        ver = int(rng.integers(0, 3))
        tps = []
        for _ in range(int(rng.integers(1, 3))):
            parts = []
            for p in range(int(rng.integers(1, 3))):
                msgs = []
                for _ in range(int(rng.integers(1, 4))):
                    msgs.append(compressed(inner(ver), ver) if rng.random() < 0.6
                                else k_message(payload(int(rng.integers(0, 200))), version=ver))
                parts.append((p, msgs))
            tps.append((topics[int(rng.integers(0, len(topics)))], parts))
        out.append(k_produce(ver, i, "client-%02d" % int(rng.integers(0, 4)), tps))
    return out


def kafka_workload(n, nconns=256, seed=None, adversarial=False, all_kinds=False):
    seed = SEED_BASE + 3 if seed is None else seed
    if all_kinds:
        reqs = kafka_all_kinds(n, seed)
    else:
        reqs = kafka_adversarial(n, seed) if adversarial else kafka_requests(n, seed)
    arena, offs, lens = pack(reqs)
    rng = np.random.default_rng(seed + 1)
    conn_ids = rng.integers(0, nconns, size=n).astype(np.uint32)
    conns = make_conns(nconns, 0, 9092, True, PROTO_KAFKA, 2000 + np.arange(nconns))
    return Workload("cfg3", arena, offs, lens, conn_ids, conns, cfg3_policy())


# ------------------------------------------------------------------ memcached
# proxylib memcached: text protocol lines
# (text/parser.go:72-198) and 24-byte-header binary packets (binary/parser.go).
MC_PORT = 11211


def mc_rules():
    """memcache.Rule maps (proxylib/memcached/parser.go:114-148) for cfg5."""
    return [
        {"command": "get", "keyPrefix": "user:"},
        {"command": "set", "keyRegex": "^session:[0-9a-f]{8}$"},
        {"command": "delete", "keyExact": "tmp"},
        {"command": "storage", "keyPrefix": "cache:"},
        {"command": "gat", "keyRegex": "^user:[0-9]+$"},
        {"command": "stats"},
        {"command": "touch", "keyRegex": "é|ü"},
        {"command": "writeGroup", "keyExact": "counter"},
    ]


def mc_policy():
    """Two groups on the memcached port (mc rules for remotes 3000-3127,
    version-only for any remote), plus a port-0 entry allowing 'noop'."""
    groups = [api.port_rule(remote_policies=list(range(3000, 3128)), l7proto="memcache", l7=mc_rules()),
              api.port_rule(l7proto="memcache", l7=[{"command": "version"}])]
    wild = [api.port_rule(l7proto="memcache", l7=[{"command": "noop"}, {"command": "flush_all"}])]
    return api.policy_set(api.network_policy("10.0.0.5", 5, ingress=[(MC_PORT, groups), (0, wild)]))


def _mc_key(rng, i):
    k = int(rng.integers(0, 10))
    if k < 4:
        return b"user:%d" % int(rng.integers(0, 100000))
    if k < 6:
        return b"session:%08x" % int(rng.integers(0, 1 << 32)) if rng.random() < 0.8 else b"session:zz%d" % i
    if k == 6:
        return b"cache:" + bytes(rng.choice(_ALNUM, size=int(rng.integers(1, 40))))
    if k == 7:
        return [b"tmp", b"counter", b"k\xc3\xa9y", b"\xfc\xfc"][int(rng.integers(0, 4))]
    return b"obj%d" % int(rng.integers(0, 1 << 20))


def mc_bin(opcode, key=b"", extras=b"", value=b"", magic=0x80, body=None):
    bl = len(extras) + len(key) + len(value) if body is None else body
    return struct.pack(">BBHBBHIIQ", magic, opcode, len(key), len(extras), 0, 0, bl, 0, 0) + extras + key + value


def memcache_requests(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    text_cmds = [b"get", b"gets", b"gat", b"gats", b"set", b"add", b"replace", b"append", b"prepend", b"cas",
                 b"delete", b"incr", b"decr", b"touch", b"stats", b"version", b"flush_all", b"quit"]
    for i in range(n):
        if rng.random() < 0.3:  # binary
            op = int(rng.choice([0, 1, 2, 4, 9, 10, 12, 13, 17, 20, 28, 16, 11, 5]))
            key = _mc_key(rng, i)
            extras = b"" if op in (0, 4, 9, 12, 13, 20, 10, 16, 11) else bytes(8)
            value = bytes(rng.integers(0, 256, size=int(rng.integers(0, 200)), dtype=np.uint8)) if op in (1, 2, 17) else b""
            out.append(mc_bin(op, b"" if op in (10, 16, 11) else key, extras, value))
            continue
        c = text_cmds[int(rng.integers(0, len(text_cmds)))]
        if c in (b"get", b"gets"):
            line = c + b" " + b" ".join(_mc_key(rng, i) for _ in range(int(rng.integers(1, 5))))
        elif c in (b"gat", b"gats"):
            line = c + b" %d " % int(rng.integers(0, 1000)) + b" ".join(_mc_key(rng, i) for _ in range(int(rng.integers(1, 4))))
        elif c in (b"set", b"add", b"replace", b"append", b"prepend", b"cas"):
            vlen = int(rng.integers(0, 600))
            line = c + b" %s %d %d %d" % (_mc_key(rng, i), int(rng.integers(0, 65536)), int(rng.integers(0, 3600)), vlen)
            if c == b"cas":
                line += b" %d" % int(rng.integers(0, 1 << 40))
            if rng.random() < 0.2:
                line += b" noreply"
            out.append(line + b"\r\n" + bytes(rng.choice(_ALNUM, size=vlen)) + b"\r\n")
            continue
        elif c in (b"delete",):
            line = c + b" " + _mc_key(rng, i) + (b" noreply" if rng.random() < 0.2 else b"")
        elif c in (b"incr", b"decr"):
            line = c + b" " + _mc_key(rng, i) + b" %d" % int(rng.integers(0, 100))
        elif c == b"touch":
            line = c + b" " + _mc_key(rng, i) + b" %d" % int(rng.integers(0, 100))
        elif c == b"flush_all":
            line = c + (b" %d" % int(rng.integers(0, 100)) if rng.random() < 0.5 else b"")
        else:
            line = c
        out.append(line + b"\r\n")
    return out


_MC_SPACES = [b" ", b"\t", b"\x0b", b"\x0c", b"\r", b"\n", b"\xc2\x85", b"\xc2\xa0", b"\xe1\x9a\x80", b"\xe2\x80\x80",
              b"\xe2\x80\x8a", b"\xe2\x80\xa8", b"\xe2\x80\xa9", b"\xe2\x80\xaf", b"\xe2\x81\x9f", b"\xe3\x80\x80"]
_MC_NOT_SPACES = [b"\xc2\x84", b"\xe2\x80\x8b", b"\xe2\x80", b"\xc2", b"\xe3\x80", b"\xff", b"\x00", b"\xe2\x82\xac",
                  b"\xed\xa0\x80", b"\xf0\x9f\x98\x80"]


def memcache_adversarial(n, seed):
    """Mutated memcached requests: Unicode / control separators, truncation,
    lone CR, empty lines, unknown and get*/gat*-prefixed commands, bad or
    huge storage lengths, short / wrapped binary headers."""
    rng = np.random.default_rng(seed)
    base = memcache_requests(n, seed + 3)
    out = []
    for r in base:
        op = int(rng.integers(0, 14))
        if r[0] >= 0x80:
            r = bytearray(r)
            if op < 3:
                r = r[: int(rng.integers(0, len(r) + 1))]
            elif op < 5 and len(r) >= 12:
                r[8:12] = struct.pack(">I", int(rng.choice([0, 0xFFFFFFE8, 0xFFFFFFF0, 0x7FFFFFFF, 5, 1 << 31])))
            elif op < 7 and len(r) >= 5:
                r[4] = int(rng.integers(0, 256))
            elif op < 8 and len(r) >= 4:
                r[2:4] = struct.pack(">H", int(rng.integers(0, 70)))
            elif op < 9:
                r[0] = int(rng.choice([0x80, 0x81, 0xFF, 0x90]))
            out.append(bytes(r))
            continue
        lf = r.find(b"\r\n")
        line, rest = r[:lf], r[lf:]
        toks = line.split(b" ")
        if op == 0:  # Unicode / control separators
            line = b"".join(t + _MC_SPACES[int(rng.integers(0, len(_MC_SPACES)))] for t in toks)
        elif op == 1:  # non-space multibyte junk glued to tokens
            line = b"".join(t + _MC_NOT_SPACES[int(rng.integers(0, len(_MC_NOT_SPACES)))] + b" " for t in toks)
        elif op == 2:  # truncation
            out.append(r[: int(rng.integers(0, len(r)))])
            continue
        elif op == 3:  # ends with a lone CR / LF
            out.append(line + rng.choice([b"\r", b"\n", b"\n\r", b""]))
            continue
        elif op == 4:  # empty / blank line
            line = [b"", b"   ", b"\t", b"\xe3\x80\x80"][int(rng.integers(0, 4))]
        elif op == 5:  # unknown or prefixed commands
            toks[0] = [b"getx", b"gatt", b"ge", b"GET", b"sets", b"foo", b"gatherall", b"lru", b"watch", b"misbehave",
                       b"cache_memlimit", b"slabs", b"lru_crawler", b"decr"][int(rng.integers(0, 14))]
            line = b" ".join(toks)
        elif op == 6 and toks[0] in (b"set", b"add", b"replace", b"append", b"prepend", b"cas"):  # bad lengths
            if len(toks) >= 5:
                toks[4] = [b"-1", b"+7", b"abc", b"", b"99999999999999999999", b"9223372036854775807", b"-9223372036854775808",
                           b"4294967290", b"-", b"+", b"007", b"-0"][int(rng.integers(0, 12))]
            line = b" ".join(toks)
        elif op == 7:  # drop trailing tokens
            line = b" ".join(toks[: int(rng.integers(1, len(toks) + 1))])
        elif op == 8:  # leading whitespace
            line = b"  " + line
        out.append(line + rest)
    return out


def memcache_workload(n, nconns=256, seed=None, adversarial=False):
    seed = SEED_BASE + 5 if seed is None else seed
    reqs = memcache_adversarial(n, seed) if adversarial else memcache_requests(n, seed)
    arena, offs, lens = pack(reqs)
    rng = np.random.default_rng(seed + 1)
    conn_ids = rng.integers(0, nconns, size=n).astype(np.uint32)
    # remotes: 3/4 inside the mc-rule group, 1/4 outside; a few on another port (port-0 entry)
    src = np.where(np.arange(nconns) % 4 != 3, 3000 + np.arange(nconns) % 128, 9000 + np.arange(nconns))
    conns = make_conns(nconns, 0, MC_PORT, True, PROTO_MEMCACHE, src)
    conns["port"][::16] = 11212
    if adversarial:  # connections whose parser (text / binary) was already chosen by earlier traffic
        conns["flags"] = rng.integers(0, 3, size=nconns)
    meta = {} if adversarial else {"payload_bytes": mc_inspected_bytes(reqs)}
    return Workload("cfg5-mc", arena, offs, lens, conn_ids, conns, mc_policy(), meta)


def mc_inspected_bytes(reqs):
    """Bytes a memcached parser reads per request: text = the command line up to
    and including its CRLF; binary = 24-byte header + extras + key."""
    tot = 0
    for r in reqs:
        if r and r[0] >= 0x80:
            tot += min(len(r), 24 + (r[4] if len(r) > 4 else 0) + (int.from_bytes(r[2:4], "big") if len(r) > 3 else 0))
        else:
            lf = r.find(b"\r\n")
            tot += len(r) if lf < 0 else lf + 2
    return tot


# ------------------------------------------------------------------ cfg5 mixed stream, tiling
def mixed_workload(n, seed=None):
    """cfg5: 50 % HTTP (cfg2 rules), 30 % Kafka (cfg3 rules), 20 % memcached,
    interleaved in one batch; three endpoint policies (HTTP, Kafka, memcached)."""
    seed = SEED_BASE + 5 if seed is None else seed
    nh, nk = n // 2, (n * 3) // 10
    nm = n - nh - nk
    h = http_workload(2, nh, seed=seed + 11)
    k = kafka_workload(nk, seed=seed + 13)
    m = memcache_workload(nm, seed=seed + 17)
    pol = {"policies": [h.policy["policies"][0], dict(k.policy["policies"][0], name="10.0.0.2"),
                        m.policy["policies"][0]]}
    conns = np.concatenate([h.conns, k.conns, m.conns])
    ch, ck = len(h.conns), len(k.conns)
    conns["policy"][ch:ch + ck] = 1
    conns["policy"][ch + ck:] = 2
    arena = np.concatenate([h.arena, k.arena, m.arena])
    offs = np.concatenate([h.offsets, k.offsets + np.uint64(len(h.arena)),
                           m.offsets + np.uint64(len(h.arena) + len(k.arena))])
    lens = np.concatenate([h.lengths, k.lengths, m.lengths])
    cids = np.concatenate([h.conn_ids, k.conn_ids + np.uint32(ch), m.conn_ids + np.uint32(ch + ck)])
    perm = np.random.default_rng(seed).permutation(len(offs))
    # repack in arrival order, the way a batch packer appends requests
    buf = arena.tobytes()
    arena2, offs2, lens2 = pack([buf[int(o):int(o) + int(l)] for o, l in zip(offs[perm], lens[perm])])
    payload = int(h.lengths.astype(np.int64).sum() + k.lengths.astype(np.int64).sum()) + m.meta["payload_bytes"]
    return Workload("cfg5", arena2, offs2, lens2, cids[perm], conns, pol, {"payload_bytes": payload})


PROTO_NAMES = {PROTO_HTTP: "http", PROTO_KAFKA: "kafka", PROTO_MEMCACHE: "memcache"}


def protocol_bytes(w):
    """Per protocol: request count and the payload bytes its classifier must
    read (every byte for HTTP and Kafka; for memcached the
    command line, or the 24-byte header + extras + key).  Algorithmic bytes
    of a protocol's kernel = payload + 25 per request."""
    proto = w.conns["proto"][np.minimum(w.conn_ids, len(w.conns) - 1)] if len(w.conns) else np.zeros(w.n, np.uint8)
    proto = np.where(w.conn_ids < len(w.conns), proto, 0)
    out = {}
    for p, name in PROTO_NAMES.items():
        sel = np.nonzero(proto == p)[0]
        if p == PROTO_MEMCACHE:
            buf = w.arena
            reqs = (bytes(buf[int(w.offsets[i]):int(w.offsets[i]) + int(w.lengths[i])]) for i in sel)
            payload = mc_inspected_bytes(reqs)
        else:
            payload = int(w.lengths[sel].astype(np.int64).sum())
        out[name] = {"requests": int(len(sel)), "payload": int(payload)}
    return out


def select(w, idx, name=None):
    """The requests idx of w repacked into a compact arena of their own (one
    rank's connection shard), in the same order."""
    idx = np.asarray(idx, np.int64)
    offs = w.offsets[idx].astype(np.int64)
    lens = w.lengths[idx].astype(np.int64)
    new_offs = np.zeros(len(idx), np.uint64)
    if len(idx) > 1:
        new_offs[1:] = np.cumsum(lens[:-1]).astype(np.uint64)
    mv = memoryview(np.ascontiguousarray(w.arena))
    arena = np.frombuffer(b"".join(mv[o:o + n] for o, n in zip(offs.tolist(), lens.tolist())), np.uint8)
    meta = {}
    return Workload(name or (w.name + "[shard]"), np.ascontiguousarray(arena), new_offs, w.lengths[idx].copy(),
                    w.conn_ids[idx].copy(), w.conns, w.policy, meta)


def tile_offsets(w, k):
    """Request metadata for k back-to-back copies of w's arena (copy j at byte
    offset j * len(arena)).  The arena itself is replicated on the device, so a
    100M-request stream needs only the unique part on the host; every copy's
    verdicts must equal the oracle's verdicts of the unique part."""
    if k == 1:
        return w.offsets, w.lengths, w.conn_ids
    shift = (np.arange(k, dtype=np.uint64) * np.uint64(len(w.arena)))[:, None]
    offs = (w.offsets[None, :] + shift).reshape(-1)
    return offs, np.tile(w.lengths, k), np.tile(w.conn_ids, k)


# ------------------------------------------------------------------ r2d2
# proxylib's example line protocol (proxylib/r2d2/r2d2parser.go): "CMD [file]\r\n"
R2D2_PORT = 4040


def r2d2_policy():
    """r2d2 rules (proxylib/r2d2/r2d2parser.go:69-107): cmd only, file only,
    both, an NFA-fallback file regex, a remote-restricted group, and a port-0
    entry."""
    rules = [{"cmd": "READ", "file": "^/pub/"}, {"cmd": "WRITE", "file": "tmp[0-9]+$"}, {"cmd": "HALT"},
             {"file": "(a|b)*a(a|b){14}"}, {"file": "é"}]
    groups = [api.port_rule(remote_policies=[7, 8], l7proto="r2d2", l7=[{"cmd": "RESET"}]),
              api.port_rule(remote_policies=list(range(100, 164)), l7proto="r2d2", l7=rules)]
    wild = [api.port_rule(l7proto="r2d2", l7=[{"cmd": "READ", "file": "^/wild"}])]
    return api.policy_set(api.network_policy("r2", 9, ingress=[(R2D2_PORT, groups), (0, wild)]))


def r2d2_requests(n, seed):
    rng = np.random.default_rng(seed)
    cmds = [b"READ", b"WRITE", b"HALT", b"RESET", b"READX", b"", b"read"]
    files = [b"/pub/a", b"/priv/b", b"tmp12", b"xtmp7", b"/wild/z", b"\xc3\xa9t\xc3\xa9", b"",
             b"ab" * 3 + b"a" + b"ab" * 7, b"bbbbbbbbbbbbbbbbbbbb"]
    out = []
    for i in range(n):
        c = cmds[int(rng.integers(0, len(cmds)))]
        f = files[int(rng.integers(0, len(files)))]
        k = int(rng.integers(0, 10))
        if k < 6:
            line = c + b" " + f
        elif k == 6:
            line = c
        elif k == 7:
            line = c + b" " + f + b" extra"
        elif k == 8:
            line = b" " + c + b" " + f if rng.random() < 0.5 else c + b"  " + f
        else:
            line = c + b" " + f + b"\rx"
        tail = b"\r\n" if rng.random() < 0.95 else (b"\r" if rng.random() < 0.5 else b"")
        out.append(line + tail)
    return out


def r2d2_workload(n, nconns=64, seed=None):
    seed = SEED_BASE + 7 if seed is None else seed
    reqs = r2d2_requests(n, seed)
    arena, offs, lens = pack(reqs)
    rng = np.random.default_rng(seed + 1)
    conn_ids = rng.integers(0, nconns, size=n).astype(np.uint32)
    remotes = [7, 8, 100, 101, 150, 163, 5] * (nconns // 7 + 1)
    conns = make_conns(nconns, 0, R2D2_PORT, True, PROTO_R2D2, remotes[:nconns])
    return Workload("r2d2", arena, offs, lens, conn_ids, conns, r2d2_policy())


# ------------------------------------------------------------------ cassandra
# proxylib's cassandra parser (proxylib/cassandra/cassandraparser.go): CQL
# native-protocol v3/v4 frames (9-byte header + body); QUERY / PREPARE carry a
# [long string] query
CASS_PORT = 9042


def cassandra_policy():
    """cassandra rules (cassandraparser.go:99-134): action only, table regex
    only, both, an NFA-fallback table regex, a table-less action, a
    remote-restricted group and a port-0 entry."""
    rules = [{"query_action": "select", "query_table": "^ks1\\."}, {"query_action": "insert", "query_table": "users$"},
             {"query_table": "^system\\.local$"}, {"query_action": "use"}, {"query_action": "create-index"},
             {"query_table": "(a|b)*a(a|b){14}"}, {"query_action": "update", "query_table": "é"},
             {"query_action": "drop-table", "query_table": "^\\.tmp"}]
    groups = [api.port_rule(remote_policies=[7, 8], l7proto="cassandra", l7=[{"query_action": "delete"}]),
              api.port_rule(remote_policies=list(range(100, 164)), l7proto="cassandra", l7=rules)]
    wild = [api.port_rule(l7proto="cassandra", l7=[{"query_action": "select", "query_table": "^wild"}])]
    return api.policy_set(api.network_policy("cs", 11, ingress=[(CASS_PORT, groups), (0, wild)]))


def cass_frame(op, body, stream=1, version=4, flags=0):
    return bytes([version, flags, (stream >> 8) & 0xFF, stream & 0xFF, op]) + len(body).to_bytes(4, "big") + body


def cass_query_frame(q, op=0x07, stream=1, trailer=b"\x00\x01\x00"):
    b = q.encode() if isinstance(q, str) else q
    return cass_frame(op, len(b).to_bytes(4, "big") + b + trailer, stream)


_CASS_QUERIES = [
    "SELECT * FROM ks1.users WHERE id = 1", "select a, b from users", "select * from system.local",
    "SELECT * FROM System.Local;", "select x from t from ks1.t2", "select * from", "select * from t -- c",
    "INSERT INTO users (a) VALUES (1)", "insert into ks2.users (a) values (1)", "insert into",
    "update ks1.t set a = 1", "UPDATE t SET b = 2", "delete from ks1.old where x = 1", "use ks1", "USE \"KS2\"",
    "use 'ks/x'", "create table if not exists ks1.t (a int)", "drop table if exists .tmp1", "drop table tmpx",
    "create index i on t (a)", "create custom index j on t (b)", "drop materialized view v",
    "truncate table ks1.t", "truncate t", "list roles", "create role r", "create a/bab c",
    "alter keyspace ks1 with x", "grant select on t to r", "select * from a/b", "select * from wildcat",
    "select * from ÉTÉ", "update été set a = 1", "SELECT * FROM \u212aS1.t", "\u0130NSERT INTO users x",
    "select\u00a0*\u00a0from\u2003ks1.a", "select * from t\udcff", "", "select",
    "select * from " + "ab" * 3 + "a" + "ab" * 7, "select * from bbbbbbbbbbbbbbbbbbbb",
]


def cassandra_requests(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        k = int(rng.integers(0, 20))
        stream = int(rng.integers(0, 65536))
        if k < 13:
            q = _CASS_QUERIES[int(rng.integers(0, len(_CASS_QUERIES)))]
            b = q.encode("utf-8", "surrogateescape")
            if rng.random() < 0.05:
                b = b.replace(b"t", b"\xff", 1)  # an invalid UTF-8 byte
            out.append(cass_query_frame(b, 0x09 if rng.random() < 0.2 else 0x07, stream))
        elif k == 13:
            out.append(cass_frame(int(rng.choice([0x01, 0x05, 0x0B, 0x0F, 0x20])), b"\x00" * int(rng.integers(0, 8)), stream))
        elif k == 14:
            out.append(cass_frame(0x0A, b"\x00\x02ab\x00\x00", stream))                  # EXECUTE
        elif k == 15:
            out.append(cass_frame(0x0D, b"\x00\x00\x01\x00\x00\x00\x00\x04use x", stream))  # BATCH: panics
        elif k == 16:
            f = cass_query_frame("select * from ks1.t", 0x07, stream)
            out.append(f[:int(rng.integers(0, len(f)))])                                    # short
        elif k == 17:
            f = bytearray(cass_query_frame("select * from ks1.t", 0x07, stream))
            f[int(rng.choice([0, 1]))] |= int(rng.choice([0x80, 0x01]))                     # reply / compressed
            out.append(bytes(f))
        elif k == 18:
            body = (1000).to_bytes(4, "big") + b"use x"                                     # query past the frame
            out.append(cass_frame(0x07, body, stream))
        else:
            out.append(bytes([4, 0, 0, 1, 7]) + (0x10000001).to_bytes(4, "big"))             # > 256 MB
    return out


def cassandra_workload(n, nconns=16, seed=None):
    seed = SEED_BASE + 9 if seed is None else seed
    reqs = cassandra_requests(n, seed)
    arena, offs, lens = pack(reqs)
    rng = np.random.default_rng(seed + 1)
    conn_ids = rng.integers(0, nconns, size=n).astype(np.uint32)
    remotes = [7, 8, 100, 101, 150, 163, 5] * (nconns // 7 + 1)
    conns = make_conns(nconns, 0, CASS_PORT, True, PROTO_CASSANDRA, remotes[:nconns])
    return Workload("cassandra", arena, offs, lens, conn_ids, conns, cassandra_policy())
