"""The Envoy C++ adapter (include/l7gpu_envoy.hpp): NetworkPolicyMap::Allowed's
shape over the batch C-ABI, driven by tests/native/envoy_adapter_main.cc on the
GPU.  The 19 Envoy integration verdicts (envoy/cilium_integration_test.cc,
tests/golden/reference_kats.json) come back through Allowed() from decoded
headers, through AllowedAsync on the asynchronous batcher (l7g_batcher, four
submitting threads), and the batched form agrees with the oracle's rule ids."""
import json
import os
import re
import subprocess

import numpy as np
import pytest

from cilium_amd import gen
from cilium_amd._lib import ALLOW, PROTO_HTTP

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "native", "bin", "envoy_adapter_main")


def decoded_headers(raw):
    """What Envoy's HTTP/1 codec hands the filter: pseudo headers + the rest."""
    head = raw.split("\r\n\r\n", 1)[0].split("\r\n")
    m, p, _ = head[0].split(" ", 2)
    hs = [(":method", m), (":path", p)]
    for line in head[1:]:
        k, v = line.split(":", 1)
        k, v = k.strip().lower(), v.strip()
        hs.append((":authority", v) if k == "host" else (k, v))
    return hs


def test_envoy_kats_through_allowed(kats, oracle):
    assert os.path.exists(EXE), "built by __graft_entry__.build() / cilium_amd.build.build_test_natives()"
    h = kats["http"]
    lines = [json.dumps(h["policy"])]
    for case in h["cases"]:
        c = case["conn"]
        remote = c["src_id"] if c["ingress"] else c["dst_id"]
        hs = decoded_headers(case["request"])
        lines.append("\t".join([c["policy_name"], "1" if c["ingress"] else "0", str(c["port"]), str(remote)] +
                               [f"{k}={v}" for k, v in hs]))
    r = subprocess.run([EXE], input="\n".join(lines) + "\n", capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    out = r.stdout.split("\n")
    n = len(h["cases"])
    batch = [tuple(int(x) for x in ln.split()) for ln in out[:n]]
    single = [int(x) for x in out[n:n + min(n, 8)]]
    k = n + min(n, 8)
    asyn = [tuple(int(x) for x in ln.split()) for ln in out[k:k + n]]
    want = [1 if case["expect"] == "ALLOW" else 0 for case in h["cases"]]
    assert [b[0] for b in batch] == want
    assert single == want[:len(single)]
    assert asyn == batch  # the batcher's verdicts and rule ids equal the synchronous batch
    # rule ids as the oracle resolves them for the same requests
    names = [p["name"] for p in h["policy"]["policies"]]
    conns = [{"policy": names.index(c["conn"]["policy_name"]) if c["conn"]["policy_name"] in names else -1,
              "port": c["conn"]["port"], "ingress": int(c["conn"]["ingress"]), "proto": PROTO_HTTP,
              "src_id": c["conn"]["src_id"], "dst_id": c["conn"]["dst_id"]} for c in h["cases"]]
    reqs = [c["request"].encode() for c in h["cases"]]
    arena, offs, lens = gen.pack(reqs)
    v, rule, _ = oracle.Policy(h["policy"]).classify(conns, arena, offs, lens, np.arange(n, dtype=np.uint32))
    assert [b[1] for b in batch] == [int(x) if y == ALLOW else -1 for x, y in zip(rule, v)]
