"""The C-ABI library loads and exports every entry point include/l7gpu.h
declares (no compute calls: those need a GPU)."""
import ctypes as C
import os
import re
import subprocess

import pytest

import cilium_amd
from cilium_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared(header):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(l7g_[a-z_]+)\s*\(", src)))


def test_library_exports_header_symbols():
    lib = _lib.load()
    names = declared("l7gpu.h") + declared("proxylib_abi.h")
    assert "l7g_classify" in names and "l7g_policy_update" in names
    for name in names:
        assert hasattr(lib, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True, text=True).stdout
    for name in names:
        assert re.search(rf"\bT {name}\b", out), name
    assert set(_lib.EXPORTS) <= set(names)


def test_library_contains_gfx950_code():
    blob = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # offload bundle entry of the HIP kernels


def test_engine_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no such HIP device"):
        cilium_amd.Engine(0)


def test_debug_regex_error_text():
    with pytest.raises(ValueError, match=r"missing argument to repetition operator: `\*`"):
        cilium_amd.debug_regex("*", b"")


def test_envoy_adapter_driver_links():
    """The C++ adapter header compiles against the C-ABI and its driver links
    libl7gpu.so (run on the GPU by tests/test_gpu_envoy_adapter.py)."""
    from cilium_amd import build
    exe = build.build_test_natives()[0]
    out = subprocess.run(["ldd", exe], capture_output=True, text=True).stdout
    assert "libl7gpu.so" in out and "not found" not in out.split("libl7gpu.so")[1].split("\n")[0]
