#!/usr/bin/env python3
"""Generate the Unicode data tables used by the Go-regexp-compatible parsers.

Two consumers, two identical copies of the same *data* (no code is shared):
  - cilium_amd/csrc/regex/unicode_tables.h   (product: regex -> DFA compiler)
  - oracle/unicode_tables.h                  (oracle: Pike-VM restatement)

What Go's regexp/syntax needs (Go 1.10.3 per the reference's
contrib/packaging/docker/Dockerfile.runtime:84, i.e. Unicode 10.0):
  * simple case-folding orbits (unicode.SimpleFold) for (?i)
  * general categories for \\pL, \\p{Lu}, ...  (unicode.Categories)
  * scripts for \\p{Greek}, ...                (unicode.Scripts)

  * simple lower-case mapping (unicode.ToLower) for proxylib cassandra's
    strings.ToLower (proxylib/cassandra/cassandraparser.go:373)

This container only has Unicode 13.0 data (Python unicodedata, Perl unicore).
The reference holds the Unicode 10.0.0 *assigned* set
(vendor/golang.org/x/text/unicode/rangetable/tables10.0.0.go, assigned10_0_0):
every table is intersected with it, so code points Unicode 11-13 assigned
(e.g. the Georgian Mtavruli capitals U+1C90-U+1CBF and their fold pairs) are
unassigned here, as in Go 1.10.  Properties of code points already assigned in
10.0 are taken from 13.0 data (changes to those are not pinned).  Scripts that
did not exist in Unicode 10.0 are dropped.  Generation runs in the build
container only (it reads /root/reference); the output is committed.
"""
import re
import os
import subprocess
import sys
import unicodedata

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MAXR = 0x10FFFF
ASSIGNED10 = os.environ.get(
    "L7G_ASSIGNED10", "/root/reference/vendor/golang.org/x/text/unicode/rangetable/tables10.0.0.go")


def load_assigned10(path=ASSIGNED10):
    """assigned10_0_0 of x/text/unicode/rangetable: R16 + R32 {lo, hi, stride}."""
    src = open(path).read()
    body = src[src.index("var assigned10_0_0 = &unicode.RangeTable{"):]
    body = body[:body.index("LatinOffset")]
    cps = set()
    for lo, hi, st in re.findall(r"\{0x([0-9a-fA-F]+), 0x([0-9a-fA-F]+), (\d+)\}", body):
        cps.update(range(int(lo, 16), int(hi, 16) + 1, int(st)))
    return cps


A10 = None  # set of code points assigned in Unicode 10.0 (main() loads it)

# Scripts added in Unicode 11.0-13.0 (absent from Go 1.10's unicode.Scripts).
POST10_SCRIPTS = {
    "Dogra", "Gunjala_Gondi", "Hanifi_Rohingya", "Makasar", "Medefaidrin",
    "Old_Sogdian", "Sogdian", "Elymaic", "Nandinagari", "Nyiakeng_Puachue_Hmong",
    "Wancho", "Chorasmian", "Dives_Akuru", "Khitan_Small_Script", "Yezidi",
}
# Perl spells some names differently from Go's unicode.Scripts keys.
SCRIPT_NAME_FIX = {
    "Nko": "Nko", "Phags_pa": "Phags_Pa", "Signwriting": "SignWriting",
}


def go_script_name(perl_name):
    parts = perl_name.split("_")
    name = "_".join(p[:1].upper() + p[1:] for p in parts)
    return SCRIPT_NAME_FIX.get(name, name)


def ranges_of(pred_codes):
    out = []
    start = prev = None
    for c in pred_codes:
        if start is None:
            start = prev = c
        elif c == prev + 1:
            prev = c
        else:
            out.append((start, prev))
            start = prev = c
    if start is not None:
        out.append((start, prev))
    return out


def simple_fold_target(c):
    ch = chr(c)
    cf = ch.casefold()
    if len(cf) == 1:
        return ord(cf)
    lo = ch.lower()
    if len(lo) == 1:
        return ord(lo)
    return c


def fold_orbits():
    parent = {}

    def find(x):
        while parent.get(x, x) != x:
            parent[x] = parent.get(parent[x], parent[x])
            x = parent[x]
        return x

    def union(a, b):
        ra, rb = find(a), find(b)
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)

    for c in range(MAXR + 1):
        if 0xD800 <= c <= 0xDFFF or c not in A10:
            continue
        t = simple_fold_target(c)
        if t != c and t in A10:
            union(c, t)
    groups = {}
    for c in list(parent.keys()):
        groups.setdefault(find(c), set()).add(c)
    for c in list(parent.values()):
        groups.setdefault(find(c), set()).add(c)
    pairs = []
    for g in groups.values():
        if len(g) < 2:
            continue
        s = sorted(g)
        for i, r in enumerate(s):
            pairs.append((r, s[(i + 1) % len(s)]))
    pairs.sort()
    return pairs


def categories():
    cats = {}
    for c in range(MAXR + 1):
        cat = unicodedata.category(chr(c))
        if cat == "Cn" or c not in A10:
            continue
        cats.setdefault(cat, []).append(c)
    out = {}
    for k, v in cats.items():
        out[k] = ranges_of(v)
    # Aggregates as in Go's unicode.Categories ("C" excludes Cn).
    for major in "CLMNPSZ":
        codes = sorted(c for k, v in cats.items() if k[0] == major for c in v)
        out[major] = ranges_of(codes)
    return out


def scripts():
    txt = subprocess.check_output(
        ["perl", "-MUnicode::UCD=charscripts", "-e",
         'my $s=charscripts(); for my $k (sort keys %$s){ print "$k";'
         ' for my $r (@{$s->{$k}}){ print " $r->[0]-$r->[1]"; } print "\\n"; }'],
        text=True)
    out = {}
    for line in txt.splitlines():
        parts = line.split()
        name = go_script_name(parts[0])
        if name in POST10_SCRIPTS or name in ("Unknown", "Zzzz"):
            continue
        codes = set()
        for p in parts[1:]:
            a, b = p.split("-")
            codes.update(range(int(a), int(b) + 1))
        merged = ranges_of(sorted(codes & A10))
        if merged:
            out[name] = merged
    return out


def simple_lower():
    """unicode.ToLower: the UnicodeData simple lower-case mapping (one rune);
    str.lower() agrees except for U+0130, whose full mapping has two runes."""
    out = []
    for c in range(MAXR + 1):
        if 0xD800 <= c <= 0xDFFF or c not in A10:
            continue
        lo = chr(c).lower()
        t = 0x69 if c == 0x130 else (ord(lo) if len(lo) == 1 else c)
        if t != c and t in A10:
            out.append((c, t))
    return out


def emit(path, pairs, cats, scr, lower):
    lines = []
    w = lines.append
    w("/* GENERATED by tools/gen_unicode.py -- do not edit.")
    w(" * Unicode %s properties (Python unicodedata + Perl Unicode::UCD) restricted to the" % unicodedata.unidata_version)
    w(" * Unicode 10.0.0 assigned set of Go 1.10 (x/text rangetable assigned10_0_0).")
    w(" * Tables for Go regexp/syntax semantics: SimpleFold orbits, categories, scripts;")
    w(" * unicode.ToLower pairs. */")
    w("#pragma once")
    w("#include <stdint.h>")
    w("")
    w("/* (rune, next rune in its simple-fold orbit), sorted by rune. */")
    w("static const uint32_t UNI_FOLD_PAIRS[][2] = {")
    for i in range(0, len(pairs), 6):
        w("  " + " ".join("{0x%X,0x%X}," % p for p in pairs[i:i + 6]))
    w("};")
    w("static const int UNI_FOLD_NPAIRS = %d;" % len(pairs))
    w("")
    allr = []
    table = []
    for kind, d in (("cat", cats), ("script", scr)):
        for name in sorted(d):
            rs = d[name]
            table.append((name, len(allr), len(rs), 0 if kind == "cat" else 1))
            allr.extend(rs)
    w("/* concatenated inclusive ranges (lo, hi) */")
    w("static const uint32_t UNI_RANGES[][2] = {")
    for i in range(0, len(allr), 6):
        w("  " + " ".join("{0x%X,0x%X}," % r for r in allr[i:i + 6]))
    w("};")
    w("typedef struct { const char *name; int off; int n; int is_script; } uni_table_t;")
    w("static const uni_table_t UNI_TABLES[] = {")
    for name, off, n, isscr in table:
        w('  {"%s", %d, %d, %d},' % (name, off, n, isscr))
    w("};")
    w("static const int UNI_NTABLES = %d;" % len(table))
    w("")
    w("/* (rune, unicode.ToLower(rune)) for every rune the mapping changes, sorted. */")
    w("static const uint32_t UNI_LOWER_PAIRS[][2] = {")
    for i in range(0, len(lower), 6):
        w("  " + " ".join("{0x%X,0x%X}," % p for p in lower[i:i + 6]))
    w("};")
    w("static const int UNI_LOWER_NPAIRS = %d;" % len(lower))
    with open(path, "w") as f:
        f.write("\n".join(lines) + "\n")


def main():
    global A10
    A10 = load_assigned10()
    pairs = fold_orbits()
    cats = categories()
    scr = scripts()
    lower = simple_lower()
    for rel in ("cilium_amd/csrc/regex/unicode_tables.h", "oracle/unicode_tables.h"):
        emit(os.path.join(ROOT, rel), pairs, cats, scr, lower)
    print("fold pairs", len(pairs), "categories", len(cats), "scripts", len(scr), "lower", len(lower),
          file=sys.stderr)


if __name__ == "__main__":
    main()
