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
    declared = set(re.findall(r"^\s*(?:int|void|int64_t|const char\*)\s+(bls_\w+)\(", hdr, re.M))
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


def test_hw_queues_requested_by_the_host_not_the_library():
    """The library never writes the environment as it loads (a load-time setenv
    races other threads' getenv and leaks into child processes); the host asks with
    bls_gpu_request_hw_queues before its first HIP call -- the Python wrapper does as it
    loads the library -- and an explicit value or $BLS_KEEP_HW_QUEUES=1 is kept.  Before
    any context, bls_admission reports the count the runtime will read (known = 2)."""
    import os
    import subprocess
    import sys

    # the C environment (os.environ is Python's snapshot from start-up)
    getenv = ("libc = ctypes.CDLL(None); libc.getenv.restype = ctypes.c_char_p; "
              "v = libc.getenv(b'GPU_MAX_HW_QUEUES'); ")
    raw = ("import ctypes; lib = ctypes.CDLL(%r); " % str(LIB_PATH)) + getenv + (
        "a = v.decode() if v else None; r = lib.bls_gpu_request_hw_queues(16); v = libc.getenv(b'GPU_MAX_HW_QUEUES'); "
        "r2 = lib.bls_gpu_request_hw_queues(8); print(a, r, v.decode() if v else None, r2)")
    wrapped = ("import ctypes, sys; sys.path.insert(0, %r); from lodestar_amd import _abi; "
               "from lodestar_amd.native import admission; _abi.load_library(); " % str(ROOT)) + getenv + (
        "a = admission(0); print(v.decode() if v else None, _abi.HW_QUEUES_REQUEST, a['hw_queues'], "
        "a['hw_queues_known'])")
    env = {k: v for k, v in os.environ.items() if k not in ("GPU_MAX_HW_QUEUES", "BLS_KEEP_HW_QUEUES")}

    def run(code, **extra):
        out = subprocess.run([sys.executable, "-c", code], env=dict(env, **extra), capture_output=True, text=True,
                             timeout=120)
        assert out.returncode == 0, out.stderr[-800:]
        return out.stdout.split()

    # loading the bare library leaves the environment alone; the request applies once
    assert run(raw) == ["None", "0", "16", "1"]
    assert run(raw, GPU_MAX_HW_QUEUES="4") == ["4", "1", "4", "1"]
    # the Python wrapper asks for 24 unless told not to
    assert run(wrapped) == ["24", "0", "24", "2"]
    assert run(wrapped, GPU_MAX_HW_QUEUES="4") == ["4", "1", "4", "2"]
    assert run(wrapped, BLS_KEEP_HW_QUEUES="1") == ["None", "None", "4", "2"]


def test_device_count_without_gpu():
    from lodestar_amd._abi import load_library

    lib = load_library()
    assert lib.bls_gpu_device_count() >= 0


def test_scratch_admission_accounting():
    """The admission arithmetic (bls_scratch_plan, no device): queues per priority level
    are min(contexts, GPU_MAX_HW_QUEUES); the per-queue figure is the deepest kernel's
    reservation from the build's resource table; a context is admitted while
    queues x per-queue <= budget (include/lodestar_bls.h bls_admission)."""
    import json

    from lodestar_amd._abi import load_library
    from lodestar_amd.native import scratch_plan

    lib = load_library()
    res = json.loads((ROOT / "lodestar_amd" / "_native" / "kernel_resources.json").read_text())
    from lodestar_amd.build import FIXTURE_KERNELS, FIXTURE_TUS, _plain_name

    # the deepest verify-path kernel (fixture and probe kernels never run on a verifier context)
    per_queue = max(k["device_scratch_bytes"] for k in res["kernels"]
                    if k["tu"] not in FIXTURE_TUS and _plain_name(k["name"]) not in FIXTURE_KERNELS)
    assert res["scratch_per_queue"] == per_queue > 0
    assert res["scratch_worst_kernel"].encode() == lib.bls_scratch_worst_kernel()
    lib.bls_gpu_set_scratch_budget(0)
    ok, a = scratch_plan(12, 1, 24)
    assert ok and a["queues_in_use"] == 13 and a["scratch_per_queue"] == per_queue
    assert a["scratch_reserved"] == 13 * per_queue and a["scratch_budget"] == 6 << 30
    # at HIP's default 4 queues per priority every context count fits
    ok, a = scratch_plan(64, 8, 4)
    assert ok and a["queues_in_use"] == 8
    # the largest admissible count with one queue per context, and one more refused
    cap = (6 << 30) // per_queue
    assert scratch_plan(cap - 1, 1, 64)[0] and not scratch_plan(cap, 1, 64)[0]
    # an override budget (bls_gpu_set_scratch_budget) moves the cap; 0 restores it
    lib.bls_gpu_set_scratch_budget(3 * per_queue)
    try:
        assert scratch_plan(2, 1, 64)[0] and not scratch_plan(3, 1, 64)[0]
    finally:
        lib.bls_gpu_set_scratch_budget(0)
    assert scratch_plan(12, 1, 24)[1]["scratch_budget"] == 6 << 30


def test_fixture_kernels_scratch_checked():
    """build.scratch_per_queue counts the verify path's kernels only and refuses a build
    whose fixture kernels (signing, probes: they run on verifier contexts' streams too)
    would need more scratch than that figure."""
    import pytest

    from lodestar_amd.build import scratch_per_queue

    table = [{"name": "_Z7k_chainv", "tu": "k_chain", "device_scratch_bytes": 100},
             {"name": "_Z6k_signv", "tu": "k_sign", "device_scratch_bytes": 90}]
    assert scratch_per_queue(table) == (100, "k_chain")
    table[1]["device_scratch_bytes"] = 101
    with pytest.raises(RuntimeError, match="fixture kernel"):
        scratch_per_queue(table)


def test_debug_flag_bits_disjoint():
    """Every BLS_DEBUG_* flag / field of include/lodestar_bls.h owns its own bits (a new
    flag once landed on BLS_DEBUG_PACK's bits), and the ctypes constants agree."""
    import lodestar_amd._abi as abi

    hdr = (ROOT / "include" / "lodestar_bls.h").read_text()
    vals = {m.group(1): int(m.group(2), 0) for m in re.finditer(r"#define (BLS_DEBUG_\w+) (0x[0-9a-fA-F]+|\d+)u", hdr)}
    masks = [v for k, v in vals.items() if not k.endswith("_MASK")] + [vals["BLS_DEBUG_PACK_MASK"],
                                                                        vals["BLS_DEBUG_MLF_PL_MASK"]]
    seen = 0
    for v in masks:
        assert seen & v == 0, hex(v)
        seen |= v
    for k, v in vals.items():
        if not k.endswith("_MASK"):
            assert getattr(abi, k[len("BLS_"):]) == v, k
