#!/usr/bin/env python3
"""Pin the algorithmic work model used for bench.py's roofline figure.

Runs the kernels' own stage bodies on the CPU (tests/native/hostsim.cpp, built with
an Fp-multiplication counter) over a cfg2-shaped batch (single-pubkey batchable
requests, chunks of 16) and records Fp Montgomery products per unit of work for
each stage.  One product = 288 v_mad_u64_u32 (12x12 limb products + 12x12
reduction products in the CIOS loop of field.hpp:fp_mul).

    python tools/work_model.py   ->  lodestar_amd/work_model.json
"""
from __future__ import annotations

import ctypes
import hashlib
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

from lodestar_amd._abi import BlsBatch, BlsStats  # noqa: E402
from lodestar_amd.build import build_hostsim  # noqa: E402
from lodestar_amd.native import pack_requests  # noqa: E402

MADS_PER_FPM = 288
STAGES = ["pk", "sig", "h2c", "scale", "miller", "status+chunk", "individual"]


def interop_sk(i: int) -> int:
    r = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
    return int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % r


def main(n: int = 64) -> None:
    lib = ctypes.CDLL(str(build_hostsim(verbose=False)))
    lib.hs_fpm_count.restype = ctypes.c_ulonglong
    lib.hs_stage_fpm.restype = ctypes.c_ulonglong
    lib.hs_verify_batch.argtypes = [ctypes.POINTER(BlsBatch), ctypes.c_void_p, ctypes.POINTER(BlsStats)]
    sks = [interop_sk(i).to_bytes(32, "big") for i in range(n)]
    pks = b""
    for sk in sks:
        o = ctypes.create_string_buffer(48)
        lib.hs_sk_to_pk(sk, o)
        pks += o.raw
    lib.hs_clear_pubkeys()
    lib.hs_load_pubkeys(pks, n, 48, None)
    reqs = []
    for i in range(n):
        m = hashlib.sha256(i.to_bytes(8, "little") + b"LODE").digest()
        o = ctypes.create_string_buffer(96)
        lib.hs_sign(sks[i], m, o)
        reqs.append((True, [([i], m, o.raw)]))
    pb = pack_requests(reqs, seed=bytes(range(32)))
    from lodestar_amd.native import _ptr  # same marshalling as the GPU path
    import numpy as np

    b = BlsBatch()
    b.n_sets, b.n_reqs = pb.n_sets, pb.n_reqs
    keep = []
    for f in ("req_set_offsets", "req_batchable", "messages", "signatures", "pubkeys", "set_pk_offsets",
              "pk_indices", "signature_lens"):
        a = getattr(pb, f)
        keep.append(a)
        setattr(b, f, _ptr(a))
    seed = ctypes.create_string_buffer(pb.seed, 32)
    b.seed = ctypes.cast(seed, ctypes.c_void_p)
    verdicts = np.zeros(n, dtype=np.int32)
    st = BlsStats()
    lib.hs_verify_batch(ctypes.byref(b), _ptr(verdicts), ctypes.byref(st))
    assert (verdicts == 1).all(), verdicts
    per = {STAGES[k]: lib.hs_stage_fpm(k) for k in range(7)}
    model = {
        "mads_per_fpm": MADS_PER_FPM,
        "batch": {"n_sets": n, "n_chunks": int(st.n_chunks), "shape": "single-pubkey batchable requests"},
        "fpm_per_set": {k: per[k] / n for k in ("pk", "sig", "h2c", "scale", "miller")},
        "fpm_per_chunk": per["status+chunk"] / max(st.n_chunks, 1),
        "note": "Fp Montgomery products counted by the host build of the kernels (tests/native/hostsim.cpp)",
    }
    model["fpm_per_set_total"] = sum(model["fpm_per_set"].values()) + model["fpm_per_chunk"] * st.n_chunks / n
    out = ROOT / "lodestar_amd" / "work_model.json"
    out.write_text(json.dumps(model, indent=1) + "\n")
    print(json.dumps(model, indent=1))


if __name__ == "__main__":
    main()
