"""proxylib access log on the GPU path: with "access-log-path" the instance
sends one protobuf cilium.LogEntry per request verdict (and per binary
memcached reply) over a unixpacket socket, as proxylib/accesslog/client.go
does; the records carry the connection's identity and the parser's L7 fields
(memcached/text/parser.go:163-196, binary/parser.go:97-137).  Records are
decoded with Google's protobuf runtime (tests/npds_pb.py descriptors)."""
import os
import socket
import struct
import tempfile

import pytest

import npds_pb
from cilium_amd import api, gen
from cilium_amd import proxylib as P

pytestmark = pytest.mark.gpu


@pytest.fixture()
def logsock():
    d = tempfile.mkdtemp()
    path = os.path.join(d, "access_log.sock")
    srv = socket.socket(socket.AF_UNIX, socket.SOCK_SEQPACKET)
    srv.bind(path)
    srv.listen(4)
    srv.settimeout(20)
    yield srv, path
    srv.close()


def read_all(conn, n):
    LE = npds_pb.cls("LogEntry")
    out = []
    for _ in range(n):
        m = LE()
        m.ParseFromString(conn.recv(65536))
        out.append(m)
    return out


def test_access_log_records(logsock):
    srv, path = logsock
    mid = P.open_module([("access-log-path", path), ("node-id", "host~127.0.0.1~alog~localdomain")])
    assert mid
    try:
        P.policy_update(mid, gen.mc_policy())
        c = P.Connection(mid, "memcache", 1001, True, 3001, 5, "1.1.1.1:5000", "10.0.0.5:11211", "10.0.0.5", 512)
        assert c.result == P.OK
        conn, _ = srv.accept()
        conn.settimeout(20)
        res, ops = c.on_data(False, [b"get user:1 user:2\r\ndelete tmp\r\nget nope\r\n"], 8)
        assert res == P.OK and [o for o, _ in ops][:3] == [P.PASS, P.PASS, P.DROP]
        recs = read_all(conn, 3)
        assert [r.entry_type for r in recs] == [0, 0, 2]  # Request, Request, Denied
        for r in recs:
            assert (r.policy_name, r.source_security_id, r.destination_security_id) == ("10.0.0.5", 3001, 5)
            assert (r.source_address, r.destination_address, r.is_ingress) == ("1.1.1.1:5000", "10.0.0.5:11211", True)
            assert r.WhichOneof("l7") == "generic_l7" and r.generic_l7.proto == "textmemcached"
            assert r.timestamp > 0
        assert dict(recs[0].generic_l7.fields) == {"command": "get", "keys": "user:1, user:2"}
        assert dict(recs[1].generic_l7.fields) == {"command": "delete", "keys": "tmp"}
        assert dict(recs[2].generic_l7.fields) == {"command": "get", "keys": "nope"}
        c.close()
        # binary: the request, then the reply
        b = P.Connection(mid, "memcache", 1002, True, 3001, 5, "1.1.1.1:5001", "10.0.0.5:11211", "10.0.0.5", 512)
        req = gen.mc_bin(0, key=b"user:7")
        res, ops = b.on_data(False, [req], 4)
        assert ops[:1] == [(P.PASS, len(req))]
        rep = gen.mc_bin(0, key=b"", value=b"v", magic=0x81)
        res, ops = b.on_data(True, [rep], 4)
        assert ops[:1] == [(P.PASS, len(rep))]
        r1, r2 = read_all(conn, 2)
        assert (r1.entry_type, r2.entry_type) == (0, 1)
        assert dict(r1.generic_l7.fields) == {"opcode": "0", "key": "user:7"} and r1.generic_l7.proto == "binarymemcached"
        b.close()
        # http: a denial carries status 403
        pol = api.policy_set(api.network_policy("web", 1, ingress=[(80, [api.port_rule(http=[{"headers": [
            {"name": ":path", "regex_match": "/ok"}]}])])]))
        P.policy_update(mid, pol)
        h = P.Connection(mid, "http", 1003, True, 9, 2, "1.1.1.1:5002", "10.0.0.9:80", "web", 1024)
        ok = b"GET /ok HTTP/1.1\r\nHost: svc\r\n\r\n"
        no = b"POST /no HTTP/1.1\r\nHOST:  other \r\n\r\n"
        res, ops = h.on_data(False, [ok + no], 4)
        assert ops[:2] == [(P.PASS, len(ok)), (P.DROP, len(no))]
        a, d = read_all(conn, 2)
        assert (a.entry_type, d.entry_type) == (0, 2) and a.WhichOneof("l7") == "http"
        assert (a.http.method, a.http.path, a.http.host, a.http.status, a.http.http_protocol) == ("GET", "/ok", "svc", 0, 1)
        assert (d.http.method, d.http.path, d.http.host, d.http.status) == ("POST", "/no", "other", 403)
        h.close()
        conn.close()
    finally:
        P.close_module(mid)
