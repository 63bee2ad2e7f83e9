import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs via gpurun)")


@pytest.fixture(scope="session")
def kats():
    with open(os.path.join(ROOT, "tests", "golden", "reference_kats.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def oracle():
    import refpy
    refpy.build()
    return refpy


@pytest.fixture(scope="session")
def engine():
    """Product engine on cuda:0 (GPU tests only).  Fails loudly without the
    HIP library or a device: there is no CPU fallback."""
    from cilium_amd import Engine
    return Engine(0)
