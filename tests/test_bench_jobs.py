"""bench.py's multi-GPU job modes, dry run on CPU (gloo, world_size 2):

  --mode cfg4     the range-sync job sharded by call (aggregates, invalid sets, the
                  non-batchable 128-set calls at reduced size);
  --mode cfg5     each rank's epoch slice (committee-shared roots, invalid sets);
  --mode sharded  --shape cfg4 / cfg5: every call split over the ranks, Fp12 partials,
                  one final exponentiation, bad-shard localisation of failing calls.

The bench's own functions (bench_job -> run_job_slice / run_sharded_job, the verdict
checks against validity by construction, the max-over-ranks reduction) run unchanged;
only the per-rank device is replaced by the oracle (test infrastructure, never the
product): OracleCtx restates bls_gpu_verify_many with oracle.verify_many_signature_sets
(worker.ts:32-108) over the same packed calls, OraclePartialBackend the shard partials.
"""
from __future__ import annotations

import argparse
import os
import socket
from types import SimpleNamespace

import numpy as np
import pytest


class OracleCtx:
    """The GpuContext calls bench_job makes, answered by the oracle on the CPU."""

    def __init__(self):
        from oracle import bls_oracle as O

        self.O = O
        self.table = []

    def sk_to_pk(self, blob: bytes) -> np.ndarray:
        O = self.O
        sks = [int.from_bytes(blob[k:k + 32], "big") for k in range(0, len(blob), 32)]
        return np.array([list(O.g1_compress(O.sk_to_pk(s))) for s in sks], dtype=np.uint8)

    def load_pubkeys(self, pks: bytes, width: int) -> np.ndarray:
        assert width == 48
        for k in range(0, len(pks), 48):
            code, pt = self.O.g1_decompress(pks[k:k + 48])
            assert code == self.O.E_OK
            self.table.append(pt)
        return np.zeros(len(pks) // 48, dtype=np.int32)

    def sign(self, sks: bytes, msgs: bytes) -> np.ndarray:
        O = self.O
        out = [O.g2_compress(O.sign(int.from_bytes(sks[32 * k:32 * k + 32], "big"), msgs[32 * k:32 * k + 32]))
               for k in range(len(sks) // 32)]
        return np.array([list(s) for s in out], dtype=np.uint8)

    def aggregate(self, idx):
        return self.O.aggregate_pubkeys([self.table[i] for i in idx])

    def _requests(self, pb):
        reqs = []
        for r in range(len(pb.req_batchable)):
            sets = []
            for i in range(int(pb.req_set_offsets[r]), int(pb.req_set_offsets[r + 1])):
                idx = pb.pk_indices[pb.set_pk_offsets[i]:pb.set_pk_offsets[i + 1]]
                n = int(pb.signature_lens[i]) if pb.signature_lens is not None else 96
                sets.append((self.aggregate([int(x) for x in idx]), pb.messages[32 * i:32 * i + 32].tobytes(),
                             pb.signatures[96 * i:96 * i + n].tobytes()))
            reqs.append((bool(pb.req_batchable[r]), sets))
        return reqs

    def verify_many(self, pbs):
        verdicts, retries, ok = [], 0, 0
        for pb in pbs:
            res, rt, good = self.O.verify_many_signature_sets(self._requests(pb))
            verdicts.append(np.array([(1 if v else 0) if kind == "success" else -v.code for kind, v in res],
                                     dtype=np.int32))
            retries += rt
            ok += good
        return verdicts, SimpleNamespace(batch_retries=retries, batch_sigs_success=ok, merged_check=0,
                                         device_ms=0.0, stage_ms=[0.0] * 8)


class OraclePartialBackend:
    """shard.GpuPartialBackend's two calls over table-index sets, by the oracle."""

    def __init__(self, ctx: OracleCtx):
        self.ctx = ctx
        self.O = ctx.O

    def partial(self, sets, base, seed):
        import hashlib

        O = self.O
        f = O.F12_ONE
        for k, (idx, msg, sig) in enumerate(sets):
            s = O.signature_from_bytes(sig, validate=True)
            r = int.from_bytes(hashlib.sha256(seed + (base + k).to_bytes(4, "little")).digest()[:8], "big") or 1
            f = O.f12_mul(f, O.miller_loop(O.E1.mul(self.ctx.aggregate(idx), r), O.hash_to_g2(msg)))
            f = O.f12_mul(f, O.miller_loop(O.E1.neg(O.G1), O.E2.mul(s, r)))
        return b"".join(v.to_bytes(48, "big") for c in f for v in c), 0, None

    def final_check(self, partials):
        O = self.O
        f = O.F12_ONE
        for p in partials:
            w = [int.from_bytes(p[48 * k: 48 * k + 48], "big") for k in range(12)]
            f = O.f12_mul(f, [(w[2 * j], w[2 * j + 1]) for j in range(6)])
        return O.f12_is_one(O.final_exponentiation(f))


def _args(**kw):
    base = dict(mode="cfg4", shape="cfg2", table_keys=16, steps=1, warmup=0, sets=4, cfg4_sets=16,
                cfg4_call_sets=8, cfg4_agg_k=4, cfg4_invalid=0.1, cfg5_sets=16, cfg5_roots=2, cfg5_call_sets=8)
    base.update(kw)
    return argparse.Namespace(**base)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


CASES = {"cfg4": dict(mode="cfg4"), "cfg5": dict(mode="cfg5"),
         "sharded_cfg4": dict(mode="sharded", shape="cfg4", cfg4_invalid=3.0),
         "sharded_cfg5": dict(mode="sharded", shape="cfg5")}


def _job_rank(rank, world, port, case, q):
    import torch.distributed as dist

    import bench

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        out = bench.bench_job(_args(**CASES[case]), [OracleCtx()], rank, world, dist, None, OraclePartialBackend)
        q.put((rank, out))
    except BaseException as e:  # noqa: BLE001 -- reported to the parent
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", list(CASES))
def test_bench_job_modes_gloo_world2(case):
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_job_rank, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=600) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in (0, 1):
        assert isinstance(res[r], dict), res[r]
        assert p.exitcode == 0
    out = res[0]
    job0, job1 = res[0]["job"], res[1]["job"]
    assert out["n_gpus"] == 2 and out["value"] > 0
    if case == "cfg4":
        # 32 sets in 4 calls of 8, two per rank; the aggregates and invalid sets of the draw
        assert job0["sets"] + job1["sets"] == 32 and job0["calls"] == job1["calls"] == 2
        assert job0["false_requests"] + job1["false_requests"] >= 1
    elif case == "cfg5":
        assert job0["sets"] == job1["sets"] == 16
        assert job0["false_requests"] >= 1 and job0["batch_retries"] >= 1
    else:
        assert job0["calls"] == 4 and job0["sets"] == 32
        if case == "sharded_cfg4":
            assert job0["failing_calls"] >= 1


def test_work_pricing_follows_pass_shape():
    """bench.py prices the roofline's algorithmic work by the pass shape the library
    reports (bls_stats.pass_shape): the Pippenger signature sum replaces the per-set
    [r] sig chains, and 1 / 2 / 4 items per k_mlf lane share f's squarings, so the
    products per set fall in that order; None keeps the environment's fixed choices."""
    import json
    from pathlib import Path

    import bench

    wm_path = Path(bench.ROOT) / "lodestar_amd" / "_native" / "work_model.json"
    if not wm_path.exists():
        pytest.skip("work model not built (build() writes it)")
    wm = json.loads(wm_path.read_text())
    assert bench.mlf_products(wm, 1 << 8) > bench.mlf_products(wm, 2 << 8) > bench.mlf_products(wm, 4 << 8)
    assert bench.mlf_products(wm, None) == wm["ml_f_pair"]
    n = 22 * 1024
    chains, _ = bench.work_per_set(n, shape=2 << 8)
    msm, note = bench.work_per_set(n, shape=1 | (2 << 8))
    quad, _ = bench.work_per_set(n, shape=1 | (4 << 8))
    assert "Pippenger" in note
    assert chains - msm > 0.8 * wm["chain_r_sig"]  # the [r] sig chains leave, the MSM costs little
    # every set's loop and the pass's one signature loop (1 / n per set) follow the shape
    assert msm - quad == pytest.approx((wm["ml_f_pair"] - wm["ml_f_quad"]) * (1 + 1 / n))
    # the per-set path's pricing follows the programs the kernel runs (one set per
    # wavefront: the |x| chains + k_pre's two GLV multiplications; packed: the r chains in
    # the programs), for every packing
    for S in (1, 2, 3):
        assert 10_000 < bench.pset_products_per_set(S) < 25_000
    small, note = bench.work_per_set(128)
    assert "k_pset" in note and small > bench.pset_products_per_set(1)


def test_bench_gpus2_launches_two_ranks():
    """`bench.py --gpus 2` with no launcher starts two rank processes itself (RANK /
    WORLD_SIZE / LOCAL_RANK, rendezvous on 127.0.0.1) and rank 0 reports n_gpus 2 -- here
    as a dry run: gloo ranks whose contexts are the oracle stand-in (--stand-in), the
    cfg4 range-sync job sharded by call at reduced size."""
    import json
    import subprocess
    import sys
    from pathlib import Path

    root = Path(__file__).resolve().parent.parent
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["PYTHONPATH"] = str(root)
    cmd = [sys.executable, str(root / "bench.py"), "--gpus", "2", "--mode", "cfg4", "--steps", "1", "--warmup", "0",
           "--inflight", "1", "--table-keys", "16", "--cfg4-sets", "16", "--cfg4-call-sets", "8", "--cfg4-agg-k", "4",
           "--cfg4-invalid", "0.1", "--stand-in", "tests.test_bench_jobs:OracleCtx"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=str(root))
    assert out.returncode == 0, out.stderr[-3000:]
    lines = out.stdout.splitlines()
    assert len(lines) == 1 and lines[0].startswith("{"), out.stdout  # rank 0's JSON line alone on stdout
    r = json.loads(lines[0])
    assert r["n_gpus"] == 2 and r["value"] > 0 and "DRY RUN" in r["data"]
    assert r["job"]["sets"] == 16 and r["job"]["calls"] == 2  # this rank's half of the 32-set job
    # a launcher's WORLD_SIZE must agree with --gpus
    bad = subprocess.run([sys.executable, str(root / "bench.py"), "--gpus", "2", "--mode", "cfg4"], capture_output=True,
                         text=True, timeout=120, env=dict(env, WORLD_SIZE="1"), cwd=str(root))
    assert bad.returncode != 0 and "WORLD_SIZE" in bad.stderr
