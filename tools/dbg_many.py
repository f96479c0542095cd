"""Debug probe: single-message sigagg calls with one invalid set, verdicts per size and
position (what tests/test_gpu_parity.py::test_verify_many_merged_signature_sum_fails
found).  Prints one line per case: size, bad index, wrong verdict indices."""
import hashlib
import sys

sys.path.insert(0, ".")
from lodestar_amd._abi import DEBUG_SIGAGG_ON, DEBUG_NO_MERGED_CHECK  # noqa: E402
from lodestar_amd.native import GpuContext, pack_requests  # noqa: E402
from oracle import bls_oracle as O  # noqa: E402


def h(b):
    return hashlib.sha256(b).digest()


gpu = GpuContext(0)
sks = [O.interop_secret_key(i).to_bytes(32, "big") for i in range(16)]
pks = gpu.sk_to_pk(b"".join(sks))
gpu.load_pubkeys(pks.tobytes(), 48)
for flags_name, flags in (("sigagg", DEBUG_SIGAGG_ON), ("sigagg_nomerged", DEBUG_SIGAGG_ON | DEBUG_NO_MERGED_CHECK),
                          ("auto", 0)):
    for n, bad in ((80, 41), (64, 41), (48, 20), (33, 5), (128, 70), (256, 130), (1024, 500), (80, 1), (80, 79)):
        msgs = [h(b"dbg%d-%d" % (n, i)) for i in range(n)]
        sigs = gpu.sign(b"".join(sks[i % 16] for i in range(n)), b"".join(msgs))
        reqs = [(True, [([i % 16], msgs[i] if i != bad else h(b"x"), sigs[i].tobytes())]) for i in range(n)]
        gpu.set_debug_flags(flags)
        v, st = gpu.verify_packed(pack_requests(reqs))
        gpu.set_debug_flags(0)
        wrong = [i for i in range(n) if int(v[i]) != (0 if i == bad else 1)]
        print(flags_name, n, bad, "wrong", wrong[:20], "merged", st.merged_check, "retries", st.batch_retries,
              flush=True)
