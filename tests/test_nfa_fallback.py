"""The bit-parallel NFA fallback at policy-compile time (CPU, host-only
engine): rule sets whose regexes exceed the DFA state budget on their own
compile -- none is rejected -- and the patterns go to the NFA pool."""
import cilium_amd
import nfa_cases


def test_blowup_rules_compile_onto_the_nfa():
    e = cilium_amd.Engine(-1)
    e.update_policy(nfa_cases.policy())
    e.set_connections(nfa_cases.conns())
    st = e.stats()
    assert st["http_nfas"] == 5  # PATH, HOST, TOKEN, INV, BIG; GET/PUT/POST and /static/.* stay DFAs
    assert st["nfa_pool_bytes"] > 0
    assert st["http_dfas"] >= 1


def test_memcache_key_regex_over_budget_compiles():
    from cilium_amd import gen
    from cilium_amd._lib import PROTO_MEMCACHE
    from test_gpu_memcache import mc_nfa_policy
    e = cilium_amd.Engine(-1)
    e.update_policy(mc_nfa_policy())
    e.set_connections(gen.make_conns(1, 0, gen.MC_PORT, True, PROTO_MEMCACHE, [1]))
    st = e.stats()
    assert st["mc_nfas"] == 3 and st["mc_rules"] == 4  # ^k:\d+$ stays a DFA
