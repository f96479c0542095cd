"""Library paths picked only by environment knobs or by a context's history, on the GPU
(ADVICE r5).  Each case runs in a fresh child process whose environment is set before
the library loads (the knobs are read once); verdicts and worker counters are checked
against the oracle's worker semantics (oracle.verify_many_signature_sets over validity
tokens, multithread/worker.ts:32-108), the pass shape against the rule that picked it.

* msm_flip (BLS_MSM=1): the Pippenger signature sum runs on a context whose last pass
  passed its merged check, and not on the pass after a failing one, which checks its
  chunks straight away (bls_gpu.hip verify_body merged_skipped, ctx->last_merged_failed):
  a failing call, then two passing ones -- pass_shape bit 0 goes 1, 0, 1, merged_check
  2, 3, 1, and every verdict is right.
* fallbacks (BLS_COOP_ML_MAX=1, BLS_INDIV2_MAX=0, BLS_PACK3_INFLIGHT=0): a failing
  aggregated call's later Miller loops above the cooperative limit take the SIMT pair at
  mlf_per_lane_alone's shape (k_pset.hip launch_k_mln_coop -> k_mlq.hip), its requests
  verified alone on one wavefront each (k_fin.hip k_indiv_coop), and a 512-set per-set
  call runs three sets per wavefront (k_pset.hip pack_for -> k_psetn<3>).
* fe_simt (BLS_FE_SIMT_MIN=1): every chunk check and every request verified alone runs
  its final exponentiation one lane per task (kernels/k_fin_simt.hip) instead of one
  wavefront per task -- failing aggregated calls (with and without group testing), the
  per-set path, non-batchable multi-set requests.
* fe_simt also sets BLS_GROUP_SUMS_MIN=0 (every group test pairs one signature sum over
  its requests' sets); gsums_off (BLS_GROUP_SUMS=0): the same calls with every
  group-tested request pairing its own signature sum; group_eq_off (BLS_GROUP_EQ=0): the
  same calls with the two-round group tests (bit groups, then the decoded request alone
  and the rest together) instead of the complement inference; group_eq_whole
  (BLS_GROUP_EQ=2): the complement inference against a test of the chunk's whole request
  list instead of the failed chunk check's own final exponentiation.
* sync_spin / sync_poll (BLS_SYNC): the host thread waits every call in
  hipStreamSynchronize's spin, or polls its event with sleeps on every call, where the
  default polls only passes of more than 2,048 sets (bls_gpu.hip pass_wait) -- the fallbacks'
  calls, verdicts unchanged.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

pytestmark = pytest.mark.gpu

ROOT = Path(__file__).resolve().parent.parent

_CHILD = r"""
import json, os, sys
sys.path.insert(0, os.environ["REPO"])
from lodestar_amd import workloads as W
from lodestar_amd.native import GpuContext, pack_requests
case = sys.argv[1]
out = {"calls": []}
with GpuContext(0) as gpu:
    K = 256
    W.load_table([gpu], K)
    sks = W.interop_sks(K)
    def make(n, tag):
        msgs = [W.message(j, tag) for j in range(n)]
        sigs = W._sign_all(gpu, [sks[j % K] for j in range(n)], msgs)
        return [([j % K], msgs[j], sigs[j]) for j in range(n)], msgs
    def run(sets, msgs, bad, batchable, per_set, flags=0):
        gpu.set_debug_flags(flags)
        s = list(sets)
        for j in bad:
            s[j] = (s[j][0], msgs[(j + 1) % len(msgs)], s[j][2])
        reqs = [(batchable, [x]) for x in s] if per_set else [(batchable, s[k:k + 128]) for k in range(0, len(s), 128)]
        v, st = gpu.verify_packed(pack_requests(reqs))
        out["calls"].append({"n": len(s), "bad": sorted(bad), "batchable": batchable, "per_set": per_set,
                             "verdicts": [int(x) for x in v], "retries": st.batch_retries, "ok": st.batch_sigs_success,
                             "shape": st.pass_shape, "merged": st.merged_check})
    if case == "msm_flip":
        sets, msgs = make(4096, b"MSMF")  # above 2,048 sets: the aggregated path
        run(sets, msgs, {17, 3500}, True, True)
        run(sets, msgs, set(), True, True)
        run(sets, msgs, set(), True, True)
    elif case in ("fe_simt", "gsums_off", "group_eq_off", "group_eq_whole"):
        sets, msgs = make(1024, b"FESI")
        run(sets, msgs, {3, 400, 401, 1000}, True, True, 8)      # chunk checks + requests alone, one lane each
        run(sets, msgs, {5, 77, 78}, True, True, 8 | 128)        # ... with group testing (products only)
        small, smsgs = make(512, b"FESP")
        run(small, smsgs, {7, 300}, True, True)                  # per-set path (f holds both pairings)
        run(small, smsgs, {7, 300}, False, False)                # non-batchable 128-set requests (k_fold groups)
        run(small, smsgs, set(), False, False, 8)                # ... on the aggregated path, all valid
    else:
        sets, msgs = make(1024, b"FALL")
        run(sets, msgs, {3, 400, 401, 1000}, True, True, 8)  # BLS_DEBUG_SIGAGG_ON: merged check fails
        small, smsgs = make(512, b"PSET")
        run(small, smsgs, {7, 300}, True, True)               # per-set path, three sets per wavefront
        run(small, smsgs, {7, 300}, False, False)             # non-batchable 128-set requests
print(json.dumps(out))
"""

ENVS = {
    "msm_flip": {"BLS_MSM": "1"},
    "fallbacks": {"BLS_COOP_ML_MAX": "1", "BLS_INDIV2_MAX": "0", "BLS_PACK3_INFLIGHT": "0"},
    "fe_simt": {"BLS_FE_SIMT_MIN": "1", "BLS_GROUP_SUMS_MIN": "0"},
    "gsums_off": {"BLS_GROUP_SUMS": "0"},
    "group_eq_off": {"BLS_GROUP_EQ": "0"},
    "group_eq_whole": {"BLS_GROUP_EQ": "2"},
    "sync_spin": {"BLS_SYNC": "spin"},
    "sync_poll": {"BLS_SYNC": "poll"},
}


def _expect(oracle, call):
    """The oracle's worker verdicts and counters over validity tokens."""
    bad = set(call["bad"])
    n = call["n"]
    if call["per_set"]:
        reqs = [(call["batchable"], [j not in bad]) for j in range(n)]
    else:
        reqs = [(call["batchable"], [j not in bad for j in range(k, min(n, k + 128))]) for k in range(0, n, 128)]

    def maybe_batch(toks):
        if not toks:
            raise oracle.BlsError(oracle.E_EMPTY_SET)
        return all(toks)

    res, retries, ok = oracle.verify_many_signature_sets(reqs, maybe_batch)
    return [(1 if r[1] else 0) if r[0] == "success" else -r[1].code for r in res], retries, ok


@pytest.mark.parametrize("case", sorted(ENVS))
def test_env_selected_paths(case, oracle):
    env = {k: v for k, v in os.environ.items() if not k.startswith("BLS_")}
    env.update(ENVS[case], REPO=str(ROOT))
    r = subprocess.run([sys.executable, "-c", _CHILD, case], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stderr[-2000:]
    calls = json.loads(r.stdout.strip().splitlines()[-1])["calls"]
    for c in calls:
        v, retries, ok = _expect(oracle, c)
        assert c["verdicts"] == v, (case, c["n"], c["bad"])
        assert (c["retries"], c["ok"]) == (retries, ok), (case, c["n"], c["bad"])
    if case == "msm_flip":
        # the Pippenger sum on the first pass; after its failed merged check the next pass
        # checks its chunks straight away (merged_check 3, no total sum, no MSM); its chunks
        # all pass, so the third is back on the merged check with the MSM
        assert [c["shape"] & 1 for c in calls] == [1, 0, 1]
        assert [c["merged"] for c in calls] == [2, 3, 1]
    elif case in ("fe_simt", "gsums_off", "group_eq_off", "group_eq_whole"):
        # the second call follows a failed merged check: its chunks are checked straight away
        assert calls[0]["merged"] == 2 and calls[1]["merged"] == 3 and calls[2]["shape"] == 0
    else:
        assert calls[0]["shape"] != 0 and calls[0]["merged"] == 2  # aggregated path, merged check failed
        assert calls[1]["shape"] == 0  # the per-set path
