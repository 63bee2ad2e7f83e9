"""Go-regexp semantics: the product's byte-DFA compiler vs the oracle's
rune-level Pike VM (two independent restatements of Go 1.10 regexp), and the
oracle vs Python's `re` on the ASCII subset where Go and Python agree.

Runs on CPU: l7g_debug_regex compiles with the product compiler and walks the
resulting tables on the host (a test hook; classification itself is GPU-only).
"""
import random
import re

import pytest

import cilium_amd as ca

CURATED = [
    ("^.el.o$", b"Hello"), ("s.*", b"ssss"), ("GET", b"GET"), ("/public/.*", b"/public/x"),
    (".*public$", b"/maybe/public"), ("(?i)k", "K".encode()), ("[^a]", b"\n"), (".", b"\n"),
    ("\\bfoo\\b", b"a foo b"), ("x*", b""), ("\\x{FFFD}", b"\xe2\x82"), ("\\x{FFFD}\\x{FFFD}", b"\xe2\x82"),
    (".", b"\xe2\x82\xac"), ("..", b"\xe2\x82\xac"), ("a{3,5}", b"aaaa"), ("(?m)^b$", b"a\nb\nc"),
    ("\\B", b"ab"), ("(a|b)*c", b"ababc"), ("\\pL+", b"h\xc3\xa9llo"), ("\\x{FFFD}", b"\xef\xbf\xbd"),
    ("[\\x{80}-\\x{10FFFF}]", b"\xff"), ("(?s).", b"\n"), ("[[:alpha:]]+", b"abc"), ("\\Q.*\\E", b".*"),
    ("a{,2}", b"a{,2}"), ("(?i)ß", "ẞ".encode()), ("\\p{Greek}+", "αβ".encode()),
    ("[^\\x00-\\x{10FFFF}]", b"a"), ("\\w+", "ſ".encode()), ("(?i)\\w", "ſ".encode()),
    ("\\x{FFFD}", b"\xed\xa0\x80"), ("...", b"\xed\xa0\x80"), ("\\x{FFFD}a", b"\xf0\x90\x80a"),
    ("^$", b""), ("\\A\\z", b""), ("a\\z", b"a\n"), ("(?m)a$", b"a\n"), ("\\b", b""), ("\\B", b""),
    ("[a-c]+?", b"abc"), ("(?U)a+", b"aa"), ("(?i:A)b", b"aB"), ("(?i)[k]", "K".encode()),
]

BAD = ["*", "a**", "a++", "(", ")", "[a", "a{2,1}", "a{1001}", "\\1", "\\8", "(?z)", "\\C", "x{2}{3}",
       "\\p{Foo}", "[[:foo:]]", "\\x{110000}", "a|*", "(?P<>a)", "(?P<a-b>c)", "[z-a]", "\\", "(?i"]


@pytest.mark.parametrize("nfa", [False, True])
@pytest.mark.parametrize("pat,data", CURATED)
def test_curated_product_vs_oracle(oracle, pat, data, nfa):
    ref = oracle.Regex(pat)
    for anchored in (True, False):
        assert ca.debug_regex(pat, data, anchored, nfa) == ref.match(data, anchored), (pat, data, anchored)


@pytest.mark.parametrize("pat", BAD)
def test_compile_errors_agree(oracle, pat):
    with pytest.raises(ValueError) as e1:
        oracle.Regex(pat)
    with pytest.raises(ValueError) as e2:
        ca.debug_regex(pat, b"", True)
    assert str(e1.value) == str(e2.value)


ATOMS = ["a", "b", "c", "/", "\\.", ".", "[ab]", "[^a]", "[a-c]", "\\d", "\\w", "\\W", "\\s", "\\b", "\\B",
         "^", "$", "é", "\\x{FFFD}", "(?i:a)", "(?s:.)", "(?m:^)", "(?m:$)", "[[:digit:]]", "\\pL", "x"]
INPUT_CHARS = [b"a", b"b", b"c", b"/", b".", b"1", b" ", b"\n", b"A", "é".encode(), b"\xff", b"\xc3",
               b"\xe2\x82", b"\xef\xbf\xbd", b"_"]


def rand_pattern(rng, depth=0):
    r = rng.random()
    if depth > 3 or r < 0.35:
        s = rng.choice(ATOMS)
    elif r < 0.6:
        s = "".join(rand_pattern(rng, depth + 1) for _ in range(rng.randint(2, 3)))
    elif r < 0.75:
        s = "(" + rand_pattern(rng, depth + 1) + "|" + rand_pattern(rng, depth + 1) + ")"
    else:
        s = "(" + rand_pattern(rng, depth + 1) + ")"
    if rng.random() < 0.3:
        s += rng.choice(["*", "+", "?", "{1,2}", "{2}", "{0,1}"])
    return s


@pytest.mark.parametrize("nfa", [False, True])
def test_random_product_vs_oracle(oracle, nfa):
    rng = random.Random(1234)
    checked = 0
    for _ in range(600):
        pat = rand_pattern(rng)
        try:
            ref = oracle.Regex(pat)
        except ValueError as e:
            with pytest.raises(ValueError) as e2:
                ca.debug_regex(pat, b"", True)
            assert str(e2.value) == str(e)
            continue
        for _ in range(6):
            data = b"".join(rng.choice(INPUT_CHARS) for _ in range(rng.randint(0, 8)))
            for anchored in (True, False):
                assert ca.debug_regex(pat, data, anchored, nfa) == ref.match(data, anchored), (pat, data, anchored)
                checked += 1
    assert checked > 3000


PY_ATOMS = ["a", "b", "c", "/", "\\.", ".", "[ab]", "[^a]", "[a-c]", "\\d", "\\w", "\\W", "\\b", "x", "[[:digit:]]"]  # no \\B: Python never matches it on ""


def test_oracle_vs_python_re_ascii(oracle):
    """ASCII-safe subset where Go and Python agree (no $, \\s, {,n}, (?i),
    Unicode classes): re.fullmatch for anchored, re.search for unanchored."""
    rng = random.Random(99)
    for _ in range(400):
        atoms = [rng.choice(PY_ATOMS) for _ in range(rng.randint(1, 5))]
        pat = "".join(a + (rng.choice(["", "", "*", "+", "?", "{1,2}"]) if a not in ("\\b", "\\B") else "")
                      for a in atoms)
        pypat = pat.replace("[[:digit:]]", "[0-9]")
        cre = re.compile(pypat.encode(), re.ASCII)
        ref = oracle.Regex(pat)
        for _ in range(8):
            data = bytes(rng.choice(b"abc/.1 xA_\n") for _ in range(rng.randint(0, 8)))
            assert ref.match(data, True) == bool(cre.fullmatch(data)), (pat, data)
            assert ref.match(data, False) == bool(cre.search(data)), (pat, data)


# Patterns whose DFA explodes (the reason the NFA fallback exists): the NFA
# agrees with the oracle's Pike VM on them, at sizes the DFA cannot reach.
BLOWUP = ["(a|b)*a(a|b){14}", "(a|b)*a(a|b){20}", ".*a.{12}", "(?s).*x[^y]{10}z", "[ab]*a[ab]{9}\\b",
          "(.*/)?api/v[0-9]+/.{8}", "(?m)^.*(a|\\x{FFFD}).{6}$"]


@pytest.mark.parametrize("pat", BLOWUP)
def test_blowup_patterns_nfa_vs_oracle(oracle, pat):
    ref = oracle.Regex(pat)
    rng = random.Random(hash(pat) & 0xFFFF)
    alphabet = [b"a", b"b", b"x", b"y", b"z", b"/", b"1", "é".encode(), b"\xe2\x82", b"\n", b" "]
    for i in range(300):
        n = rng.randint(0, 40)
        data = b"".join(rng.choice(alphabet) for _ in range(n))
        if i % 3 == 0:
            data = b"api/v1/" + data
        for anchored in (True, False):
            assert ca.debug_regex(pat, data, anchored, nfa=True) == ref.match(data, anchored), (pat, data, anchored)


# Past 1,024 positions the NFA keeps sparse follow rows and its state sets in
# scratch (regex/nfa_walk.h nfa_run_big): every repeat count Go accepts.
LARGE = [".{1000}x.{1000}", "(a|b)*a.{1000}b.{1000}", "(?m)^a.{1000}.{30}$", "\\b[ab]{1000}[ab]{100}\\b",
         "(?s).{1000}.{25}\u00e9", "(x|y.{600}){1}z[^a]{500}.{400}"]


def _large_inputs(pat, rng):
    yield b""
    for _ in range(24):
        n = rng.choice([1000, 1030, 1099, 1100, 1101, 1500, 2000, 2001, 2002, 2003, 2100, 2500, 3200])
        alphabet = [b"a", b"b", b"x", b"y", b"z", b"c", b" ", b"\n", "\u00e9".encode()]
        data = bytearray(b"".join(rng.choice(alphabet[:3] if rng.random() < 0.5 else alphabet) for _ in range(n)))
        if rng.random() < 0.5 and len(data) > 1001:  # a planted x / b at the distance the pattern wants
            k = rng.randrange(0, len(data) - 1001)
            data[k] = ord("a")
            data[k + 1001] = ord(rng.choice("xb"))
        yield bytes(data)


@pytest.mark.parametrize("pat", LARGE)
def test_large_nfa_vs_oracle(oracle, pat):
    ref = oracle.Regex(pat)
    rng = random.Random(sum(pat.encode()))
    for data in _large_inputs(pat, rng):
        for anchored in (True, False):
            assert ca.debug_regex(pat, data, anchored, nfa=True) == ref.match(data, anchored), (pat, len(data), anchored)


# Unicode version of Go 1.10 (Unicode 10.0.0): the tables are restricted to the
# assigned10_0_0 set the reference vendors
# (vendor/golang.org/x/text/unicode/rangetable/tables10.0.0.go:5739), so code
# points Unicode 11-13 assigned are unassigned (Cn) and fold with nothing.
UNICODE10 = [
    # Georgian Mtavruli (Unicode 11): no category, no (?i) pair with Mkhedruli
    ("\\p{Lu}", "Ა", False), ("\\PL", "Ა", True), ("\\p{Georgian}", "Ა", False),
    ("(?i)ა", "Ა", False), ("(?i)ა", "ა", True), ("(?i)Ა", "ა", False),
    ("[^\\pL\\pM\\pN\\pP\\pS\\pZ\\pC]", "Ჿ", True),
    # Syriac Supplement (Unicode 10): assigned Lo
    ("\\p{Lo}", "ࡠ", True), ("\\p{Syriac}", "ࡪ", True), ("\\p{Lo}", "࡫", False),
    # Unicode 10 additions stay (Masaram Gondi U+11D00), Unicode 11 ones go (Dogra U+11800)
    ("\\p{Lo}", "\U00011D00", True), ("\\p{Lo}", "\U00011800", False),
    ("\\p{Masaram_Gondi}", "\U00011D00", True),
]


@pytest.mark.parametrize("nfa", [False, True])
@pytest.mark.parametrize("pat,text,want", UNICODE10)
def test_unicode10_tables(oracle, pat, text, want, nfa):
    data = text.encode()
    assert oracle.Regex(pat).match(data, True) == want, (pat, text)
    assert ca.debug_regex(pat, data, True, nfa) == want, (pat, text)


def test_unicode10_unknown_script():
    # scripts Unicode 11+ introduced do not exist in Go 1.10's unicode.Scripts
    with pytest.raises(ValueError):
        ca.debug_regex("\\p{Dogra}", b"", True)
