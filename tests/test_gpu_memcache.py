"""memcached parity on the GPU: product vs oracle, bit-exact
(SURVEY.md §8(a) P3-P6)."""
import numpy as np
import pytest

from cilium_amd import api, gen
from cilium_amd._lib import ALLOW, DENY, INCOMPLETE, PARSE_ERROR, PROTO_MEMCACHE

from test_gpu_http import assert_same, both, wl_from_reqs
from test_oracle_kats import memcache_policy

pytestmark = pytest.mark.gpu

VERDICT = {"ALLOW": ALLOW, "DENY": DENY, "INCOMPLETE": INCOMPLETE, "PARSE_ERROR": PARSE_ERROR}


def test_memcache_kats(engine, oracle, kats):
    M = kats["memcache"]
    c = M["conn"]
    for case in M["cases"]:
        pol = memcache_policy(M, case["l7_rules"])
        conns = gen.make_conns(1, 0, c["port"], c["ingress"], PROTO_MEMCACHE, [c["src_id"]], c["dst_id"])
        reqs = [bytes.fromhex(M["requests"][k["request"]]) for k in case["checks"]]
        w = wl_from_reqs(reqs, pol, conns)
        got, ref = both(engine, oracle, w, 1)
        for i, k in enumerate(case["checks"]):
            assert got[0][i] == VERDICT[k["expect"]], (case["name"], k)
            assert got[2][i] == k["consumed"], (case["name"], k)
        assert_same(got, ref, w)


def test_cfg5_memcache_parity(engine, oracle):
    w = gen.memcache_workload(30000)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    v = got[0]
    assert (v == ALLOW).mean() > 0.1 and (v == DENY).mean() > 0.1
    assert len(set(got[1].tolist())) >= 8


def test_memcache_adversarial_parity(engine, oracle):
    w = gen.memcache_workload(30000, seed=4242, adversarial=True)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    assert set(got[0].tolist()) >= {ALLOW, DENY, INCOMPLETE, PARSE_ERROR}


def test_memcache_many_rules_and_dfas(engine, oracle):
    """> 64 rules (several mask chunks) and regexes that split into several DFAs."""
    rules = []
    for k in range(150):
        m = k % 5
        if m == 0:
            rules.append({"command": "get", "keyExact": f"user:{k}"})
        elif m == 1:
            rules.append({"command": "storage", "keyPrefix": f"cache:{k % 7}"})
        elif m == 2:
            rules.append({"command": "get", "keyRegex": f"^session:[0-9a-f]{{{k % 9 + 1}}}(x|y)*{k}$"})
        elif m == 3:
            rules.append({"command": "delete", "keyRegex": f"(a|b)*a(a|b){{{k % 6 + 3}}}"})
        else:
            rules.append({"command": "writeGroup"} if k == 149 else {"command": "gat", "keyPrefix": f"user:{k}"})
    pol = api.policy_set(api.network_policy("mc", 1, ingress=[(gen.MC_PORT, [api.port_rule(l7proto="memcache", l7=rules)])]))
    base = gen.memcache_workload(20000, seed=99)
    rng = np.random.default_rng(5)
    extra = []
    for i in range(4000):
        k = int(rng.integers(0, 150))
        key = [b"user:%d" % k, b"cache:%d%d" % (k % 7, i), b"session:%s%d" % (b"ab12cdef0"[: k % 9 + 1], k),
               b"ab" * (k % 5) + b"a" + b"ab"[i % 2:] * (k % 6 + 3), b"zz"][k % 5]
        cmd = [b"get", b"set", b"get", b"delete", b"gat 5"][k % 5]
        tail = b" 0 0 1\r\nx\r\n" if cmd == b"set" else b"\r\n"
        extra.append(cmd + b" " + key + tail)
    reqs = [bytes(base.arena[int(o):int(o) + int(L)]) for o, L in zip(base.offsets, base.lengths)] + extra
    conns = gen.make_conns(4, 0, gen.MC_PORT, True, PROTO_MEMCACHE, [1, 2, 3, 4])
    w = wl_from_reqs(reqs, pol, conns, np.arange(len(reqs)) % 4)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    st = engine.stats()
    assert st["mc_dfas"] >= 2 and st["mc_rules"] == 150
    assert len(set(got[1].tolist())) > 40


def test_mixed_http_kafka_memcache_batch(engine, oracle):
    """cfg5 shape: one batch with HTTP, Kafka and memcached connections interleaved."""
    h = gen.http_workload(2, 5000)
    k = gen.kafka_workload(3000)
    m = gen.memcache_workload(2000)
    pol = {"policies": [h.policy["policies"][0], dict(k.policy["policies"][0], name="10.0.0.2"),
                        m.policy["policies"][0]]}
    conns = np.concatenate([h.conns, k.conns, m.conns])
    nh, nk = len(h.conns), len(k.conns)
    conns["policy"][nh:nh + nk] = 1
    conns["policy"][nh + nk:] = 2
    arena = np.concatenate([h.arena, k.arena, m.arena])
    offs = np.concatenate([h.offsets, k.offsets + np.uint64(len(h.arena)),
                           m.offsets + np.uint64(len(h.arena) + len(k.arena))])
    lens = np.concatenate([h.lengths, k.lengths, m.lengths])
    cids = np.concatenate([h.conn_ids, k.conn_ids + np.uint32(nh), m.conn_ids + np.uint32(nh + nk)])
    perm = np.random.default_rng(2).permutation(len(offs))
    w = gen.Workload("mixed3", arena, offs[perm], lens[perm], cids[perm], conns, pol)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)


def test_memcache_port_entries(engine, oracle):
    """proxylib port semantics (policymap.go:113-236): unknown parser => port
    not installed, no entry => deny, no L7 rules => allow, port-0 fallback,
    remote filtering, unparsed rules after an unknown parser."""
    P = api.port_rule
    pol = api.policy_set(api.network_policy("mc", 1, ingress=[
        (100, [P(l7proto="memcache", l7=[{"command": "get"}]), P(l7proto="no.such.parser", l7=[{"file": "x"}])]),
        (101, [P(remote_policies=[7])]),
        (102, [P(l7proto="memcache", l7=[{"command": "set"}]), P(remote_policies=[8], l7proto="memcache", l7=[])]),
        (103, [P(http=[{}])]),
        (104, [P(l7proto="no.such.parser", l7=[{}]), P(l7proto="memcache", l7=[{"keyExact": "no-command"}])]),
        (105, [P(l7proto="memcache", l7=[{"command": "nosuch"}])]),
        (0, [P(remote_policies=[9], l7proto="memcache", l7=[{"command": "delete"}])]),
    ]))
    reqs = [b"get a\r\n", b"set a 0 0 1\r\nx\r\n", b"delete a\r\n", b"stats\r\n", b"\x80\x00\x00\x01" + bytes(20) + b"k"]
    ports = [100, 101, 102, 103, 104, 105, 106]
    srcs = [7, 8, 9]
    conns = gen.make_conns(len(ports) * len(srcs), 0, 0, True, PROTO_MEMCACHE, 0)
    for i, (p, s) in enumerate((p, s) for p in ports for s in srcs):
        conns["port"][i], conns["src_id"][i] = p, s
    allr = [r for _ in range(len(conns)) for r in reqs]
    cids = np.repeat(np.arange(len(conns)), len(reqs))
    w = wl_from_reqs(allr, pol, conns, cids)
    got, ref = both(engine, oracle, w, 1)
    assert_same(got, ref, w)
    assert set(got[0].tolist()) == {ALLOW, DENY}


def test_cfg5_mixed_tiled_parity(engine, oracle):
    """bench.py's cfg5 stream (gen.mixed_workload, repacked in arrival order) and
    its tiling: every copy of the arena gets the oracle's verdicts of the unique part."""
    w = gen.mixed_workload(12000)
    got1, ref = both(engine, oracle, w)
    assert_same(got1, ref, w)
    offs, lens, cids = gen.tile_offsets(w, 3)
    got = engine.classify(np.tile(w.arena, 3), offs, lens, cids)
    for g, r in zip(got, ref):
        assert np.array_equal(np.asarray(g).reshape(3, -1), np.broadcast_to(np.asarray(r).reshape(1, -1), (3, w.n)))
    assert w.algorithmic_bytes() < int(w.lengths.astype(np.int64).sum()) + 25 * w.n


def mc_nfa_policy():
    rules = [{"command": "get", "keyRegex": "(a|b)*a(a|b){14}"},
             {"command": "delete", "keyRegex": "x[^y]{12}z"},
             {"command": "get", "keyRegex": "^k:\\d+$"},
             {"command": "set", "keyRegex": "é(.){10}$"}]
    return api.policy_set(api.network_policy("mc", 1, ingress=[(gen.MC_PORT, [api.port_rule(l7proto="memcache", l7=rules)])]))


def mc_nfa_requests(n, seed):
    rng = np.random.default_rng(seed)

    def ab(k, hit):
        s = bytearray(rng.choice([ord("a"), ord("b")], size=k).astype(np.uint8).tobytes())
        if k >= 15:
            s[-15] = ord("a") if hit else ord("b")
        return bytes(s)

    reqs = []
    for i in range(n):
        kind = i % 5
        if kind == 0:
            keys = [b"pre" + ab(int(rng.integers(10, 30)), bool(rng.integers(0, 2))) for _ in range(int(rng.integers(1, 4)))]
            reqs.append(b"get " + b" ".join(keys) + b"\r\n")
        elif kind == 1:
            mid = rng.choice(list(b"abyz"), size=int(rng.integers(10, 14))).astype(np.uint8).tobytes()
            reqs.append(b"delete x" + mid + b"z\r\n")
        elif kind == 2:
            reqs.append(b"get k:%d" % i + (b" " + ab(20, True) if i % 3 else b"") + b"\r\n")
        elif kind == 3:
            key = "é".encode() + rng.choice(list(b"ab\xc3\xa9"), size=int(rng.integers(8, 14))).astype(np.uint8).tobytes()
            reqs.append(b"set " + key + b" 0 0 1\r\nx\r\n")
        else:  # binary GET (opcode 0)
            reqs.append(gen.mc_bin(0, key=ab(int(rng.integers(14, 24)), bool(rng.integers(0, 2)))))
    return reqs


def test_memcache_nfa_fallback_parity(engine, oracle):
    """keyRegex patterns over the DFA budget (Go regexp.Match, unanchored) run
    as bit-parallel NFAs at each key's end; every key must match."""
    reqs = mc_nfa_requests(6000, 11)
    conns = gen.make_conns(2, 0, gen.MC_PORT, True, PROTO_MEMCACHE, [1, 2])
    w = wl_from_reqs(reqs, mc_nfa_policy(), conns, np.arange(len(reqs)) % 2)
    got, ref = both(engine, oracle, w)
    assert_same(got, ref, w)
    assert engine.stats()["mc_nfas"] >= 2
    assert len(set(got[1][got[0] == ALLOW].tolist())) == 4
    assert (got[0] == DENY).sum() > 500
