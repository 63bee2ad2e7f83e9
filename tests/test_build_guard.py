"""The product library cannot carry experiment switches: the
build refuses -D defines for libl7gpu.so, and no kernel source keeps a
verdict-changing experiment branch."""
import glob
import os
import re

import pytest

from cilium_amd import build as b

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_product_build_refuses_defines():
    with pytest.raises(ValueError):
        b.build(defines=("-DL7G_KAFKA_WIN=8",))


def test_no_experiment_switches_in_sources():
    pat = re.compile(r"L7G_\w*EXP\w*")
    hits = []
    for f in glob.glob(os.path.join(ROOT, "cilium_amd", "csrc", "**", "*"), recursive=True):
        if f.endswith((".hip", ".h", ".cc")):
            for i, line in enumerate(open(f, encoding="utf-8", errors="replace"), 1):
                if pat.search(line):
                    hits.append(f"{os.path.relpath(f, ROOT)}:{i}")
    assert not hits, hits
