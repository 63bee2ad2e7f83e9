"""The generated Unicode tables (tools/gen_unicode.py) checked against data the
generator does not read, so a generator bug is not common-mode between the
product (cilium_amd/csrc/regex/unicode_tables.h) and the oracle
(oracle/unicode_tables.h), which share the generated data.

- Categories: Python's Unicode 3.2 database (unicodedata.ucd_3_2_0, a separate
  data set from the 13.0 one the generator reads).  Every code point assigned
  in 3.2 whose category 13.0 did not change is in exactly its category's table
  and its major class's table (Go's unicode.Categories, which Go 1.10 builds
  from Unicode 10.0; 3.2 assignments are stable through 10.0).
- Simple folding: the orbits are Go's unicode.SimpleFold cycles (each rune's
  pair is the next larger rune of its orbit, wrapping to the smallest), and a
  rune with a one-rune lower-case mapping shares its orbit with it.
- unicode.ToLower pairs: sorted, unique, never identity, and inverse to the
  orbits (a rune and its lower case fold together).
"""
import os
import re
import unicodedata

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PRODUCT = os.path.join(ROOT, "cilium_amd", "csrc", "regex", "unicode_tables.h")
ORACLE = os.path.join(ROOT, "oracle", "unicode_tables.h")


def _array(text, name):
    m = re.search(r"%s\[\]\[2\] = \{(.*?)\n\};" % name, text, re.S)
    return [(int(a, 16), int(b, 16)) for a, b in re.findall(r"\{0x([0-9A-F]+),0x([0-9A-F]+)\}", m.group(1))]


@pytest.fixture(scope="module")
def tables():
    text = open(PRODUCT).read()
    ranges = _array(text, "UNI_RANGES")
    tabs = {}
    for name, off, n, is_script in re.findall(r'\{"(\w+)", (\d+), (\d+), (\d)\}', text):
        tabs[(name, int(is_script))] = ranges[int(off):int(off) + int(n)]
    return {"fold": _array(text, "UNI_FOLD_PAIRS"), "lower": _array(text, "UNI_LOWER_PAIRS"), "tabs": tabs}


def _member_set(rs):
    s = set()
    for lo, hi in rs:
        s.update(range(lo, hi + 1))
    return s


def test_product_and_oracle_hold_the_same_data():
    strip = lambda t: re.sub(r"/\*.*?\*/", "", t, flags=re.S)  # noqa: E731
    assert strip(open(PRODUCT).read()) == strip(open(ORACLE).read())


def test_categories_against_unicode_3_2(tables):
    cats = {name: _member_set(rs) for (name, script), rs in tables["tabs"].items() if not script}
    old = unicodedata.ucd_3_2_0
    checked = 0
    for c in range(0x110000):
        ch = chr(c)
        cat = old.category(ch)
        if cat == "Cn" or unicodedata.category(ch) != cat:
            continue
        checked += 1
        assert c in cats[cat], (hex(c), cat)
        assert c in cats[cat[0]], (hex(c), cat[0])
        for other, members in cats.items():
            if len(other) == 2 and other != cat:
                assert c not in members, (hex(c), cat, other)
    assert checked > 700  # 748 pairs of Unicode 3.200


def test_ranges_sorted_and_disjoint(tables):
    for key, rs in tables["tabs"].items():
        assert all(lo <= hi for lo, hi in rs), key
        assert all(hi < lo2 for (_, hi), (lo2, _) in zip(rs, rs[1:])), key


def _orbits(pairs):
    nxt = dict(pairs)
    assert len(nxt) == len(pairs)
    orbit_of = {}
    for r in nxt:
        if r in orbit_of:
            continue
        cyc = [r]
        x = nxt[r]
        while x != r:
            assert x in nxt and len(cyc) < 8, hex(r)
            cyc.append(x)
            x = nxt[x]
        o = frozenset(cyc)
        for y in cyc:
            orbit_of[y] = o
    return nxt, orbit_of


def test_fold_orbits_are_simplefold_cycles(tables):
    nxt, orbit_of = _orbits(tables["fold"])
    for r, n in nxt.items():
        o = sorted(orbit_of[r])
        assert len(o) >= 2
        i = o.index(r)
        assert n == o[(i + 1) % len(o)], (hex(r), [hex(x) for x in o])


def test_lower_case_pairs_fold_together(tables):
    _, orbit_of = _orbits(tables["fold"])
    old = unicodedata.ucd_3_2_0
    checked = 0
    for c in range(0x110000):
        ch = chr(c)
        if old.category(ch) == "Cn":
            continue
        lo = ch.lower()
        if len(lo) != 1 or lo == ch or old.category(lo) == "Cn":
            continue
        checked += 1
        assert c in orbit_of and ord(lo) in orbit_of[c], (hex(c), hex(ord(lo)))
    assert checked > 700  # 748 pairs of Unicode 3.2


def test_tolower_pairs(tables):
    lower = tables["lower"]
    _, orbit_of = _orbits(tables["fold"])
    assert [r for r, _ in lower] == sorted({r for r, _ in lower})
    for r, lo in lower:
        assert r != lo
        assert chr(r).lower() == chr(lo) or r == 0x130, hex(r)
        assert r == 0x130 or ord(chr(lo)) in orbit_of.get(r, ()), hex(r)
