#!/usr/bin/env python3
"""Benchmark of the MI355X BLS signature-set verifier (BASELINE.json metric:
"BLS signature sets verified/sec (1-8 GPUs) + p50 latency @128-set batch").

Workload per step (BASELINE.json configs[1], cfg2): one verifyManySignatureSets call of
1024 gossip-attestation sets, each its own batchable single-pubkey request (as
multithread/index.ts:260-275 buffers them), pubkeys resident in the device table
(index2pubkey, pubkeyCache.ts:56-77), random-scalar batch verification in chunks of
16 requests (worker.ts:17,56) -- every stage (decompress + subgroup check,
hash_to_G2, scalar muls, Miller loops, final exponentiations) runs inside the timed
step.  Inputs are synthetic: interop keys sk_i = LE(sha256(LE32(i))) mod r
(state-transition/src/util/interop.ts:19-22), messages sha256(LE64(j) || "LODE"),
signatures made on the GPU before timing.

Multi-GPU (torchrun, one process per GPU): each rank verifies its own 1024 sets (shard
by request, no data-path collective: scaling "weak"); value = all ranks' sets / max
over ranks of the timed region.

Also reported: p50 latency of one non-batchable 128-set call (cfg1 shape), the
roofline of the dominant kernel against the measured v_mad_u64_u32 peak, and the CPU
baseline (the oracle, rank 0, N = 1 only, bounded sample).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import statistics
import sys
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# One HIP stream per in-flight batch; HIP maps streams onto GPU_MAX_HW_QUEUES hardware
# queues (default 4 on this image), and streams sharing a queue serialise.  Give the
# in-flight contexts their own queues (set before the HIP runtime initialises; the
# box exports 4, so raise it rather than default it).
# 16 batches over 24 queues measured best (tools/gpu_inflight_q.sh: 12/16 384k,
# 16/24 403k, 20/24 382k sets/s).
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
STAGE_NAMES = ["h2d", "k_pk", "k_pre", "k_pset", "k_exact", "-", "k_status+k_chunk", "k_indiv"]
X_ABS = 0xD201000000010000
MADS_PER_FPM = 288   # 12x12 limb products + 12x12 reduction products per Montgomery product


def pset_products_per_set() -> float:
    """Expected Fp products k_pset executes per set (program MUL ops from
    lodestar_amd/_native/coop_programs.json; r's bits are uniform)."""
    pg = json.loads((ROOT / "lodestar_amd" / "_native" / "coop_programs.json").read_text())
    m = {k: v["mul_ops"] for k, v in pg.items()}
    n = m["pset_prep"] + m["pset_dbl_r"] + 0.5 * m["pset_add_r"] + 63 * m["pset_dbl_all"]
    for i in range(62, -1, -1):
        if (X_ABS >> i) & 1:
            n += 0.5 * m["pset_add_xr"] + 0.5 * m["pset_add_x"]
        else:
            n += 0.5 * m["pset_add_r"]
    return n + m["pset_phase2"] + m["pset_norm2"] + m["pset_affine2"] + m["pset_ml2"]


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary
    (profiles/*_pmc_traffic.json, written by tools/pmc_traffic.py from rocprofv3
    FETCH_SIZE / WRITE_SIZE passes of this bench), or None."""
    files = sorted((ROOT / "profiles").glob("*_pmc_traffic.json"), key=lambda p: p.name)
    for p in reversed(files):
        d = json.loads(p.read_text())
        if kernel in d:
            return int(d[kernel]["hbm_bytes_per_launch"]), p.name
    return None, None


def interop_sk(i: int) -> bytes:
    v = int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER
    return v.to_bytes(32, "big")


def make_workload(gpu, n_sets: int, rank: int, roots: int = 0):
    """cfg2: every set signs its own root.  roots > 0: the cfg5 mainnet-epoch shape
    (SURVEY §8d), consecutive sets in committees sharing `roots` signing roots per call."""
    from lodestar_amd.native import pack_requests

    n_keys = n_sets
    sks = b"".join(interop_sk(i) for i in range(n_keys))
    pks = gpu.sk_to_pk(sks)
    codes = gpu.load_pubkeys(pks.tobytes(), 48)
    assert (codes == 0).all()
    msgs = [hashlib.sha256((rank * n_sets + j).to_bytes(8, "little") + b"LODE").digest() for j in range(n_sets)]
    if roots > 0:
        msgs = [msgs[(j * roots // n_sets) * (n_sets // roots)] for j in range(n_sets)]
    sigs = gpu.sign(b"".join(interop_sk(j % n_keys) for j in range(n_sets)), b"".join(msgs))
    sets = [([j % n_keys], msgs[j], sigs[j].tobytes()) for j in range(n_sets)]
    batch = pack_requests([(True, [s]) for s in sets])
    call128 = pack_requests([(False, sets[:128])])
    return batch, call128, sets


def _oracle_batch(args) -> float:
    """One worker of the CPU baseline: build `n` sets with the oracle, then time
    verifySignatureSetsMaybeBatch over them (seconds)."""
    from oracle import bls_oracle as O

    n, base = args
    sks = [int.from_bytes(interop_sk(base + i), "big") for i in range(n)]
    msgs = [hashlib.sha256((base + j).to_bytes(8, "little") + b"LODE").digest() for j in range(n)]
    sigs = [O.g2_compress(O.sign(s, m)) for s, m in zip(sks, msgs)]
    pks = [O.sk_to_pk(s) for s in sks]
    t0 = time.perf_counter()
    ok = O.verify_signature_sets_maybe_batch(list(zip(pks, msgs, sigs)))
    dt = time.perf_counter() - t0
    assert ok
    return dt


def cpu_baseline(sample_sets: int = 16, procs: int = 16) -> dict:
    """Oracle (pure-Python restatement, oracle/bls_oracle.py) timed on the host:
    `procs` processes (the box's CPU share is 16 cores), each verifying its own
    random-scalar batch of `sample_sets` sets; value = all sets / the slowest worker's
    verification time (input construction is outside the timed part)."""
    import multiprocessing as mp

    procs = max(1, min(procs, os.cpu_count() or 1))
    with mp.get_context("spawn").Pool(procs) as pool:
        times = pool.map(_oracle_batch, [(sample_sets, 1000 * k) for k in range(procs)])
    total = sample_sets * procs
    return {"value": round(total / max(times), 3), "unit": "sets/s", "cores": procs, "kind": "port",
            "sample": f"{procs} processes x {sample_sets} single-pubkey sets, one random-scalar batch each "
                      f"(verifySignatureSetsMaybeBatch), slowest {max(times):.1f} s, pure-Python oracle"}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=96)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", type=int, default=1024)
    ap.add_argument("--latency-runs", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inflight", type=int, default=16, help="batches in flight per GPU (contexts/streams)")
    ap.add_argument("--roots", type=int, default=0,
                    help="distinct signing roots per call (0: all distinct, cfg2; 2: the cfg5 committee shape)")
    ap.add_argument("--no-dedup", action="store_true", help="hash every set's root (BLS_DEBUG_NO_MSG_DEDUP)")
    ap.add_argument("--no-merged-check", action="store_true",
                    help="one final exponentiation per chunk only (BLS_DEBUG_NO_MERGED_CHECK)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl")

    def barrier_sync():
        if dist is not None:
            import torch

            dist.barrier()
            torch.cuda.synchronize()

    from lodestar_amd.native import GpuContext

    # `inflight` verifier contexts (one HIP stream each) fed by one host thread each:
    # batches overlap on the GPU the way the reference's worker pool keeps several
    # verifyManySignatureSets jobs in flight (multithread/index.ts:199-233).
    ctxs = [GpuContext(local_rank) for _ in range(args.inflight)]
    gpu = ctxs[0]
    works = [make_workload(c, args.sets, rank, args.roots) for c in ctxs]
    from lodestar_amd._abi import DEBUG_NO_MERGED_CHECK, DEBUG_NO_MSG_DEDUP

    flags = (DEBUG_NO_MSG_DEDUP if args.no_dedup else 0) | (DEBUG_NO_MERGED_CHECK if args.no_merged_check else 0)
    for c in ctxs:
        c.set_debug_flags(flags)
    batch, call128, _ = works[0]

    for c, w in zip(ctxs, works):
        for _ in range(args.warmup):
            v, _ = c.verify_packed(w[0])
            assert (v == 1).all(), "warm-up verification failed"

    stage_sum = np.zeros(8)
    stage_n = [0]
    failures = []
    lock = threading.Lock()
    share = [args.steps // args.inflight + (1 if i < args.steps % args.inflight else 0) for i in range(args.inflight)]

    def worker(i):
        for _ in range(share[i]):
            v, st = ctxs[i].verify_packed(works[i][0])
            if not (v == 1).all():
                failures.append(i)
            with lock:
                stage_sum[:] += np.array(st.stage_ms[:])
                stage_n[0] += 1

    threads = [threading.Thread(target=worker, args=(i,)) for i in range(args.inflight)]
    barrier_sync()
    t0 = time.perf_counter()
    for t in threads:
        t.start()
    for t in threads:
        t.join()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    if failures:
        raise SystemExit("verification failed inside the timed region")
    from lodestar_amd.shard import global_throughput

    value, elapsed = global_throughput(args.sets * args.steps, elapsed, dist, device=f"cuda:{local_rank}")

    # p50 latency of one 128-set non-batchable call (cfg1 shape)
    lat = []
    for _ in range(args.latency_runs):
        t1 = time.perf_counter()
        v, _ = gpu.verify_packed(call128)
        lat.append((time.perf_counter() - t1) * 1e3)
        assert v[0] == 1

    # roofline of the dominant kernel, k_pset (VALU integer multiply-add bound).
    # stage_ms: per batch while batches overlap (a launch waits for CUs the other
    # streams hold); the roofline uses the kernel's solo launch time: the same batch
    # on one stream with the device otherwise idle (HIP events on that stream).
    stage_ms = stage_sum / max(stage_n[0], 1)
    dom = "k_pset"
    solo = []
    for _ in range(5):
        _, st = gpu.verify_packed(batch)
        solo.append(st.stage_ms[STAGE_NAMES.index(dom)])
    dom_ms = statistics.median(solo)
    shared_ms = stage_ms[STAGE_NAMES.index(dom)]
    fpm_set = pset_products_per_set()
    mads = fpm_set * MADS_PER_FPM * args.sets
    achieved = mads / (dom_ms * 1e-3) / 1e12
    peak_rate, _ = gpu.mad_peak()
    traffic, traffic_src = pmc_traffic("k_psetn" if args.sets >= 512 else "k_pset")
    peak = peak_rate / 1e12

    if rank == 0:
        out = {
            "metric": "BLS signature sets verified/sec (1-8 GPUs) + p50 latency @128-set batch",
            "value": round(value, 2),
            "unit": "sets/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u32 (381-bit Fp, 12x32-bit Montgomery limbs)",
            "data": "synthetic: interop keys, sha256 messages, GPU-made signatures",
            "config": {"workload": ("cfg2: 1024 single-pubkey gossip sets per GPU, batchable requests, "
                                    "random-scalar batch in chunks of 16 requests") if args.roots == 0 else
                                   (f"cfg5 shape: {args.sets} single-pubkey sets per call over {args.roots} "
                                    f"committee-shared signing roots, batchable requests"
                                    + (", root dedup off" if args.no_dedup else ""))
                                   + (", merged check off" if args.no_merged_check else ""),
                       "sets_per_step_per_gpu": args.sets, "inflight_batches_per_gpu": args.inflight,
                       "parallelism": f"shard-by-request x{world}"},
            "p50_latency_ms_128": round(statistics.median(lat), 3),
            "stage_ms": {k: round(float(x), 3) for k, x in zip(STAGE_NAMES, stage_ms)},
            "roofline": {"bound": "valu", "kernel": dom, "achieved": round(achieved, 4), "peak": round(peak, 3),
                         "unit": "TMAD/s (v_mad_u64_u32)", "frac": round(achieved / peak, 5), "traffic": traffic,
                         "traffic_unit": "HBM bytes/launch (PMC FETCH_SIZE x2 + WRITE_SIZE, "
                                         f"{traffic_src})" if traffic else None,
                         "work": f"{fpm_set:.0f} Fp products/set x {MADS_PER_FPM} MAD x {args.sets} sets "
                                 f"per launch, {dom_ms:.3f} ms/launch (HIP events, median of 5 solo launches "
                                 f"on one stream; {shared_ms:.3f} ms while {args.inflight} batches overlap)",
                         "device_achieved": round(value * fpm_set * MADS_PER_FPM / 1e12, 4),
                         "device_frac": round(value * fpm_set * MADS_PER_FPM / 1e12 / peak, 5),
                         "device_note": "whole-job sets/s x k_pset MADs per set: the device-wide useful "
                                        "MAD rate of the per-set kernel"},
        }
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    for c in ctxs:
        c.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
