"""The C-ABI library builds in-tree, loads without a GPU, and exports every symbol
include/lodestar_bls.h declares (no compute calls here)."""
from __future__ import annotations

import ctypes
import re
from pathlib import Path

from lodestar_amd._abi import LIB_PATH, SYMBOLS

ROOT = Path(__file__).resolve().parent.parent


def test_header_symbols_exported():
    hdr = (ROOT / "include" / "lodestar_bls.h").read_text()
    declared = set(re.findall(r"^\s*(?:int|void|int64_t|const char\*)\s+(bls_gpu_\w+)\(", hdr, re.M))
    assert declared == set(SYMBOLS)
    lib = ctypes.CDLL(str(LIB_PATH))
    for name in declared:
        assert hasattr(lib, name), name


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    """With the library absent the product path raises instead of computing on the CPU."""
    import lodestar_amd._abi as abi

    monkeypatch.setattr(abi, "LIB_PATH", tmp_path / "missing.so")
    monkeypatch.setattr(abi, "_LIB", None)
    import pytest

    with pytest.raises(RuntimeError):
        abi.load_library()


def test_device_count_without_gpu():
    from lodestar_amd._abi import load_library

    lib = load_library()
    assert lib.bls_gpu_device_count() >= 0
