"""Scratch admission on the GPU (bls_gpu_init_priority, include/lodestar_bls.h
bls_admission): contexts are opened until the library refuses one with
BLS_ERR_ADMISSION -- a clean error, no queue abort -- and every context it admitted then
verifies a call.  The reference's pool likewise keeps the workers that started and
records the one that failed (multithread/index.ts:221-229)."""
from __future__ import annotations

import hashlib

import pytest

pytestmark = pytest.mark.gpu


def test_admission_refuses_cleanly_and_admitted_contexts_verify(gpu, golden, oracle):
    from lodestar_amd._abi import load_library
    from lodestar_amd.native import AdmissionError, GpuContext, admission, pack_requests, scratch_plan

    lib = load_library()
    now = admission(0)
    per, hwq = now["scratch_per_queue"], now["hw_queues"]
    if now["contexts_normal"] + 2 >= hwq:
        pytest.skip(f"{now['contexts_normal']} normal contexts already open with {hwq} hardware queues")
    # a budget with room for exactly two more normal-priority queues
    lib.bls_gpu_set_scratch_budget(per * (now["queues_in_use"] + 2))
    opened = []
    try:
        expected = 0
        while scratch_plan(now["contexts_normal"] + expected + 1, now["contexts_high"])[0]:
            expected += 1
        assert expected == 2
        refused = None
        for _ in range(expected + 1):
            try:
                opened.append(GpuContext(0))
            except AdmissionError as e:
                refused = str(e)
                break
        assert len(opened) == expected
        assert refused is not None and refused.startswith("BLS_ERR_ADMISSION") and "GPU_MAX_HW_QUEUES" in refused
        assert admission(0)["contexts_normal"] == now["contexts_normal"] + expected
        # the refused init left nothing behind: a high-priority context is still refused too
        with pytest.raises(AdmissionError):
            GpuContext(0, high_priority=True)
        # every admitted context verifies a call
        sk = oracle.interop_secret_key(0).to_bytes(32, "big")
        msg = hashlib.sha256(b"admission").digest()
        sig = gpu.sign(sk, msg)[0].tobytes()
        pk48 = bytes.fromhex(golden["kat2_interop_pubkeys"][0])
        for c in opened:
            assert (c.load_pubkeys(pk48, 48) == 0).all()
            v, _ = c.verify_packed(pack_requests([(False, [([0], msg, sig)])]))
            assert v.tolist() == [1]
    finally:
        for c in opened:
            c.close()
        lib.bls_gpu_set_scratch_budget(0)
    assert admission(0)["contexts_normal"] == now["contexts_normal"]
    # with the default budget a context opens again
    c = GpuContext(0)
    c.close()
