"""Shared pytest fixtures.

Markers:
  gpu  -- needs a real MI355X (runs through the C-ABI library); everything else runs
          on CPU: the oracle against the reference's known-answer data, the host
          logic, and the kernels' math compiled for the CPU (tests/native/hostsim.cpp).
"""
from __future__ import annotations

import ctypes
import json
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

GOLDEN = json.loads((ROOT / "tests" / "golden" / "golden.json").read_text())


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X GPU (HIP library on cuda:0)")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def golden():
    return GOLDEN


@pytest.fixture(scope="session")
def oracle():
    from oracle import bls_oracle

    return bls_oracle


@pytest.fixture(scope="session")
def coop_programs():
    """Every cooperative program (tools/gen_coop.py build_all), generated once per session
    for the simulators of test_circuits.py and test_pset.py (~3 min)."""
    root = Path(__file__).resolve().parent.parent / "tools"
    if str(root) not in sys.path:
        sys.path.insert(0, str(root))
    import gen_coop

    progs, consts = gen_coop.build_all()
    return {p.name: p for p in progs}, consts


@pytest.fixture(scope="session")
def hostsim():
    from lodestar_amd.build import build_hostsim
    from lodestar_amd._abi import BlsBatch, BlsStats

    lib = ctypes.CDLL(str(build_hostsim(verbose=False)))
    lib.hs_verify_batch.argtypes = [ctypes.POINTER(BlsBatch), ctypes.c_void_p, ctypes.POINTER(BlsStats)]
    lib.hs_g1_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hs_g2_mul_u64.argtypes = [ctypes.c_char_p, ctypes.c_uint64, ctypes.c_char_p]
    lib.hs_fpm_count.restype = ctypes.c_ulonglong
    lib.hs_load_pubkeys.restype = ctypes.c_longlong
    return lib


@pytest.fixture(scope="session")
def gpu():
    """One GpuContext on device 0 for the whole GPU session (fails loudly without the library)."""
    from lodestar_amd.native import GpuContext

    ctx = GpuContext(0)
    yield ctx
    ctx.close()
