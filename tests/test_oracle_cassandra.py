"""The cassandra oracle (oracle/cassandra_ref.c) against the reference's own
cases (proxylib/cassandra/cassandraparser_test.go:79-282, transcribed in
tests/golden/reference_kats.json "cassandra"), plus parseQuery cases derived
by reading proxylib/cassandra/cassandraparser.go:368-469 (labelled: no
reference test asserts them, parity unpinned beyond the KATs)."""
import numpy as np
import pytest

from cilium_amd import api
from cilium_amd.engine import conns_array

import refpy

MORE, PASS, DROP, INJECT, ERROR = 0, 1, 2, 3, 4
PROTO_CASSANDRA = 5


def kat_policy(name, rule, remotes=(1, 3, 4), port=80, policy_id=2):
    return api.policy_set(api.network_policy(name, policy_id, ingress=[
        (port, [api.port_rule(remote_policies=list(remotes), l7proto="cassandra", l7=[rule])])]))


def conn_for(policy, name, port=80, src=1, dst=2):
    return conns_array([(policy.names.get(name, -1), port, 1, PROTO_CASSANDRA, src, dst)])


def op_loop(parser, bufs, max_ops=16):
    """connection.go OnData (:118-174) over one call's buffers: ops until MORE,
    an error, or the ops slice is full; returns (ops, inject bytes, log kinds)."""
    data = b"".join(bufs)
    ops, inject, logs = [], b"", []
    while len(ops) < max_ops:
        op, n, rule, path, inj = parser.request(data)
        if op == parser.PANIC:
            return "PARSER_ERROR", ops, inject, logs
        ops.append([op, n])
        inject += inj
        if op in (PASS, DROP):
            if path is not None and len(path.split(b"/")) == 4:
                logs.append(op)
            data = data[n:]
        elif op == MORE:
            break  # (an ERROR op neither advances nor stops the loop)
    return "OK", ops, inject, logs


def test_cassandra_kats(kats):
    K = kats["cassandra"]
    assert len(K["cases"]) == 7
    cc = K["connection"]
    for c in K["cases"]:
        rule = c["l7_rule"] or {"query_action": "select"}
        pol = refpy.Policy(kat_policy(c["policy_name"] if c["l7_rule"] else "cp-other", rule))
        conn = conn_for(pol, c["policy_name"], cc["port"], cc["src_id"], cc["dst_id"])
        parser = refpy.Cassandra(pol, conn)
        res, ops, inject, logs = op_loop(parser, [bytes.fromhex(b) for b in c["data"]])
        assert res == "OK", c["name"]
        assert ops == c["ops"], (c["name"], ops)
        assert inject == bytes.fromhex(c["inject"]), c["name"]
        if c["logs"] is not None:  # (passes, drops) of query-like paths
            assert [logs.count(PASS), logs.count(DROP)] == c["logs"], c["name"]


def test_kat_query_path(kats):
    K = kats["cassandra"]
    st = refpy.Cassandra()
    rc, action, table = st.parse_query(K["query"])
    assert rc == 0 and b"/query/" + action + b"/" + table == K["path"].encode()


# Derived from cassandraparser.go:368-469 (not asserted by any reference test).
# (keyspace before, query, (status, action, table) or status) ; status 1 =
# invalid (action ""), 2 = Go panic.
DERIVED = [
    ("", "SELECT * FROM ks.t", (0, "select", "ks.t")),
    ("", "select * from t;", (0, "select", ".t")),                       # TrimRight(";"), keyspace "" + "."
    ("ks", "select * from t", (0, "select", "ks.t")),
    ("ks", "select a from b from c", (0, "select", "ks.c")),            # the last FROM wins
    ("", "select * from", 2),                                            # fields[i+1] out of range
    ("", "select a from b from", 2),
    ("", "select *", 1),                                                 # no table
    ("", "SELECT -- x FROM t", 1),                                       # comment token
    ("", "select * from t /* x */", 1),
    ("", "select * from //t", 1),
    ("", "select", 1),                                                   # fewer than 2 fields
    ("", "insert into t (a) values (1)", (0, "insert", ".t")),
    ("", "insert into", 1),
    ("ks", "UPDATE T set a=1", (0, "update", "ks.t")),
    ("", "use \"KS\"", (0, "use", "ks")),                               # Trim of " \ '
    ("", "use '\\x'", (0, "use", "x")),
    ("", "CREATE TABLE IF NOT EXISTS k.t (a int)", (0, "create-table", "k.t")),
    ("", "create table if", 1),
    ("", "drop table if exists t", (0, "drop-table", ".t")),
    ("", "drop keyspace if exists k", (0, "drop-keyspace", ".k")),
    ("", "alter table if x", (0, "alter-table", ".if")),                # IF handled for create / drop only
    ("", "create keyspace k with x", (0, "create-keyspace", ".k")),
    ("", "truncate t", (0, "truncate-t", "")),                          # the truncate special case never fires
    ("", "truncate table t", (0, "truncate-table", ".t")),
    ("", "create materialized view v as", (0, "create-materialized-view", "")),
    ("", "drop custom index i", (0, "create-index", "")),
    ("", "create index i on t", (0, "create-index", "")),
    ("", "list roles", (0, "list-roles", "")),
    ("", "grant role r to s", 1),
    ("", "create a/b c", (0, "create-a/b", "")),
    ("", "select x from a/b", (0, "select", ".a/b")),
    ("", "SELECT * FROM Key.T", (0, "select", "key.t")),          # Kelvin sign -> k
    ("", "İNSERT İNTO T", (0, "insert", ".t")),              # U+0130 -> i
    ("", "select * from t", (0, "select", ".t")),                  # U+00A0 is a space
    ("", "select * from ÉTÀ", (0, "select", ".étà")),
]


@pytest.mark.parametrize("ks,query,want", DERIVED)
def test_parse_query_derived(ks, query, want):
    st = refpy.Cassandra()
    if ks:
        assert st.parse_query("use " + ks)[0] == 0
    rc, action, table = st.parse_query(query)
    if isinstance(want, int):
        assert rc == want, (query, rc, action, table)
    else:
        assert (rc, action.decode(), table.decode()) == want, (query, rc, action, table)


def test_lowering_invalid_utf8():
    """Go 1.10 strings.Map: an invalid byte before the first rune that ToLower
    changes stays raw, after it it becomes U+FFFD (derived, unpinned)."""
    st = refpy.Cassandra()
    assert st.parse_query(b"select * from t\xff")[2] == b".t\xff"                 # nothing changes: raw
    assert st.parse_query(b"SELECT * from t\xff")[2] == b".t\xef\xbf\xbd"        # 'S' changed first
    assert st.parse_query(b"select * from \xffT")[2] == b".\xfft"                  # before the change: raw


def test_use_persists_and_prepare_sets_keyspace():
    pol = refpy.Policy(kat_policy("cpx", {"query_table": "^ks2\\."}))
    conn = conn_for(pol, "cpx")
    st = refpy.Cassandra(pol, conn)

    def frame(op, body, stream=1):
        return bytes([4, 0, 0, stream, op]) + len(body).to_bytes(4, "big") + body

    def query(q, op=7, stream=1):
        b = q.encode()
        return frame(op, len(b).to_bytes(4, "big") + b + b"\x00\x01\x00", stream)

    assert st.request(query("select * from t"))[0] == DROP             # ".t"
    assert st.request(query("use ks2"))[0] == DROP                      # table "ks2": no dot for ^ks2\.
    assert st.keyspace == b"ks2"
    assert st.request(query("select * from t"))[0] == PASS              # "ks2.t"
    assert st.request(query("use ks3", op=9, stream=7))[0] == DROP      # PREPARE also sets the keyspace
    assert st.keyspace == b"ks3"
    # EXECUTE before a RESULT/prepared reply: unprepared message, ERROR INVALID_FRAME_TYPE
    ex = frame(0x0A, b"\x00\x02ab\x00\x00")
    op, n, rule, path, inj = st.request(ex)
    assert (op, n) == (ERROR, 2) and inj[11:13] == b"\x25\x00" and inj[13:] == b"\x00\x02ab"
    # RESULT kind 4 (prepared) for stream 7 binds id "ab" to the PREPARE's path
    res = bytes([0x84, 0, 0, 7, 8]) + (10).to_bytes(4, "big") + (4).to_bytes(4, "big") + b"\x00\x02ab" + b"\x00\x00"
    assert st.reply(res) == (PASS, len(res))
    op, n, rule, path, inj = st.request(ex)
    assert op == DROP and path == b"/execute/use/ks3"
    # BATCH always panics (Uint16 of a 1-byte slice)
    assert st.request(frame(0x0D, b"\x00\x00\x01\x00"))[0] == st.PANIC
    # a short QUERY body panics; a reply-direction frame is INVALID_FRAME_TYPE
    assert st.request(frame(7, b"\x00\x00"))[0] == st.PANIC
    assert st.request(bytes([0x84]) + query("use x")[1:])[:2] == (ERROR, 2)


def test_batch_api_keyspace_in_order():
    """ref_classify answers a batch's cassandra requests in order with one
    keyspace per connection (the batch-API contract, include/l7gpu.h)."""
    pol = refpy.Policy(kat_policy("cpb", {"query_table": "^a\\."}))
    conns = conns_array([(0, 80, 1, PROTO_CASSANDRA, 1, 2), (0, 80, 1, PROTO_CASSANDRA, 3, 2)])

    def q(s):
        b = s.encode()
        body = len(b).to_bytes(4, "big") + b
        return bytes([4, 0, 0, 1, 7]) + len(body).to_bytes(4, "big") + body

    reqs = [q("select * from t"), q("use a"), q("select * from t"), q("select * from t"), q("use b"),
            q("select * from t")]
    cid = np.array([0, 0, 0, 1, 0, 0], np.uint32)
    from cilium_amd import gen
    arena, offs, lens = gen.pack(reqs)
    v, r, c = pol.classify(conns, arena, offs, lens, cid)
    ALLOW, DENY = 1, 0
    assert v.tolist() == [DENY, DENY, ALLOW, DENY, DENY, DENY]
    assert c.tolist() == [len(x) for x in reqs]


def test_keyspace_with_nul_bytes():
    """Go strings hold any byte: a USE whose query runs on past its frame
    (capacity-bounded slice of the joined input) takes a keyspace token with
    NUL bytes in it, and the next table is that token + "." + table; the rule
    regex sees every byte of it (the oracle once cut the path at the first NUL
    as a C string; found by the device framing test, tests/test_gpu_frame.py)."""
    pol = refpy.Policy(kat_policy("cpn", {"query_action": "insert", "query_table": "users$"}))
    conns = conns_array([(0, 80, 1, PROTO_CASSANDRA, 1, 2)])

    def q(s, ql=None):
        b = s.encode()
        body = (len(b) if ql is None else ql).to_bytes(4, "big") + b
        return bytes([4, 0, 0, 1, 7]) + len(body).to_bytes(4, "big") + body

    use = q("use x", ql=100)  # the query is the next 100 bytes of the input
    ins = q("insert into users x")
    pad = q("select * from t") * 8
    stream = use + ins + pad
    # each request handed the input from its start to the end, as proxylib does
    offs = np.array([0, len(use)], np.uint64)
    lens = np.array([len(stream), len(stream) - len(use)], np.uint32)
    arena = np.frombuffer(stream, np.uint8).copy()
    v, r, c = pol.classify(conns, arena, offs, lens, np.zeros(2, np.uint32))
    assert c.tolist() == [len(use), len(ins)]
    assert v.tolist()[1] == 1  # keyspace "x\x04\x00...": the table still ends in "users"
