#!/usr/bin/env python3
"""Benchmark of the MI355X BLS signature-set verifier (BASELINE.json metric:
"BLS signature sets verified/sec (1-8 GPUs) + p50 latency @128-set batch").

Workload (BASELINE.json configs[1], cfg2): verifyManySignatureSets calls of 1024
gossip-attestation sets, each its own batchable single-pubkey request (as
multithread/index.ts:260-275 buffers them), pubkeys resident in the device table
(index2pubkey, pubkeyCache.ts:56-77), random-scalar batch verification in chunks of
16 requests (worker.ts:17,56); every stage (decompress + subgroup check, hash_to_G2,
scalar muls, Miller loops, final exponentiations) runs inside the timed region.
Inputs are synthetic: interop keys sk_i = LE(sha256(LE32(i))) mod r
(state-transition/src/util/interop.ts:19-22), messages sha256(LE64(j) || "LODE"),
signatures made on the GPU before timing.

A step is one call on each of the `--inflight` verifier contexts (one HIP stream
each), i.e. inflight x 1024 sets: the contexts start together (a barrier) and each
runs exactly `--steps` calls back to back, as the reference's worker pool keeps one
message per worker in flight (multithread/index.ts:199-233).  value = all sets / the
timed region, so it is steady-state whatever --steps is.

Multi-GPU (torchrun, one process per GPU):
  --mode cfg2 (default): each rank verifies its own calls (shard by request, no
      data-path collective; scaling "weak"); value = all ranks' sets / max rank time.
  --mode sharded: cfg4/cfg5 shape -- ONE call of (sets x world) sets split across
      the ranks (lodestar_amd.shard.verify_call_sharded): per rank an Fp12 partial of
      its shard, an all-gather of 588-byte records over RCCL/xGMI, one final
      exponentiation; a step is one such call.  --shape cfg4 / cfg5: four calls of the
      cfg4 mix (aggregates of --cfg4-agg-k keys, invalid sets) or of committee-shared
      roots, each split over the ranks, failing calls localised to their bad shards
      inside the timed region.
  --mode cfg4 / cfg5: BASELINE configs 4 and 5 sharded by call -- rank r verifies
      calls c with c % world == r of the range-sync job (--cfg4-sets per GPU, 1 %
      invalid, 128-set non-batchable calls) or its own epoch slice (--cfg5-sets over
      --cfg5-roots committee roots, 1024-set batchable calls, invalid sets); no
      data-path collective; verdicts checked every pass.
  --mode napi: the same cfg2 workload driven through the N-API addon and the JS
      GpuBlsVerifier (integration/js), one verifySignatureSets([set], {batchable})
      per set, as gossip validation calls it (N = 1 only).

Also reported: p50 latency of one non-batchable 128-set call (cfg1 shape), the
roofline of the dominant kernel against the measured v_mad_u64_u32 peak, and the CPU
baseline (the C++ restatement under oracle/cpu on the host cores, rank 0, N = 1).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import platform
import shutil
import statistics
import subprocess
import sys
import tempfile
import threading
import time
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))
# One HIP stream per in-flight batch; HIP maps streams onto GPU_MAX_HW_QUEUES hardware
# queues (default 4 on this image), and streams sharing a queue serialise.  Give the
# in-flight contexts their own queues (set before the HIP runtime initialises).
# (--hwq-child: the deployable-configuration sub-record runs under the queue count its
# parent gave it, HIP's default 4 included)
if "--hwq-child" not in sys.argv and int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"

R_ORDER = 0x73EDA753299D7D483339D80809A1D80553BDA402FFFE5BFEFFFFFFFF00000001
STAGE_NAMES = ["h2d", "k_pk", "k_pre", "k_chain", "sig_sums", "miller_loops", "k_status+k_chunk", "k_indiv"]
X_ABS = 0xD201000000010000
MADS_PER_FPM = 288   # 12x12 limb products + 12x12 reduction products per Montgomery product
METRIC = "BLS signature sets verified/sec (1-8 GPUs) + p50 latency @128-set batch"


def pack_of(n_sets: int) -> int:
    """Sets per wavefront k_pset runs for a call of n_sets (kernels/k_pset.hip pack_for)."""
    forced = int(os.environ.get("BLS_PACK", "0") or 0)
    if forced in (1, 2, 3):
        return forced
    return 2 if n_sets >= int(os.environ.get("BLS_PACK_MIN", "512")) else 1


def pset_products_per_set(S: int) -> float:
    """Expected Fp products the per-set kernel executes per set with S sets per
    wavefront (program MUL ops from lodestar_amd/_native/coop_programs.json): the |x|
    chains, phase 2 and the two-pair Miller loop, shared by the wavefront's S sets, plus
    k_pre's two GLV multiplications for RG and RP (work_model.json chain_r_pk each)."""
    pg = json.loads((ROOT / "lodestar_amd" / "_native" / "coop_programs.json").read_text())
    wm = json.loads((ROOT / "lodestar_amd" / "_native" / "work_model.json").read_text())
    m = {k: v["mul_ops"] for k, v in pg.items()}
    p = "pset_" if S == 1 else f"pset{S}_"
    n = m[p + "prep"] + 63 * m[p + "dbl_all"] + sum(m[p + "add_x"] for i in range(63) if (X_ABS >> i) & 1)
    n += m[p + "phase2"] + m[p + "norm2"] + m[p + "affine2"] + m[p + "ml2"]
    return n / S + 2 * wm["chain_r_pk"]


SIGAGG_MIN_SETS = 512   # bls_gpu.hip use_sigagg: the aggregated-signature path from this call size on
PERSET_MAX_INFLIGHT = 20480  # ... while more sets than this are in flight, or the call has more than
PERSET_MAX_CALL = 2048       # ... this many sets


def sigagg_of(n_sets: int, in_flight: int | None = None) -> bool:
    e = os.environ.get("BLS_SIGAGG")
    if e not in (None, ""):
        return e != "0"
    return n_sets >= SIGAGG_MIN_SETS and (n_sets > PERSET_MAX_CALL or (
        in_flight if in_flight is not None else n_sets) > PERSET_MAX_INFLIGHT)


def mlf_products(wm: dict, shape: int | None) -> float:
    """Fp products per item of k_mlf for a pass shape (items per lane in bits 8-15 of
    bls_stats.pass_shape: 1, 2 or 4 pairs share f's squarings, 3 one pair over two lanes --
    the products of one pair per f, the duplicated f.c1 l3 term not counted; None = 2)."""
    per_lane = (shape >> 8) & 0xFF if shape is not None else 2
    key = {1: "ml_f_one", 3: "ml_f_one", 4: "ml_f_quad"}.get(per_lane, "ml_f_pair")
    return wm.get(key, wm["ml_f_pair"])


def work_per_set(n_sets: int, reqs_per_chunk: int = 16, shape: int | None = None) -> tuple[float, str]:
    """Fp products the GPU executes per set for a cfg2 call of n_sets single-set
    batchable requests, every kernel of the call (k_pre, the per-set path, the chunks'
    signature sums and Miller loops, the merged check's product tree and final
    exponentiation): stage counts from lodestar_amd/_native/work_model.json
    (tools/work_model.cpp, host-compiled product math with the Fp-product counter) and
    the cooperative programs' MUL ops (coop_programs.json).  `shape`: the library's
    bls_stats.pass_shape of the timed passes (bit 0 Pippenger signature sum, bits 8-15
    items per k_mlf lane); None = the environment's fixed choices."""
    pg = json.loads((ROOT / "lodestar_amd" / "_native" / "coop_programs.json").read_text())
    wm = json.loads((ROOT / "lodestar_amd" / "_native" / "work_model.json").read_text())
    m = {k: v["mul_ops"] for k, v in pg.items()}
    chunks = max(1, n_sets // reqs_per_chunk)
    merged = (n_sets + chunks - 1) * m["fin_fmul"] + m["fin_fe1"] + m["fin_fe2"]
    # the library's pass shape says which path ran (0: the per-set path, chosen for calls
    # of >= 512 sets too while few sets are in flight, bls_gpu.hip use_sigagg)
    if (shape != 0) if shape is not None else sigagg_of(n_sets):
        # a set's Miller loop: k_mlq lines + k_mlf f side (1, 2 or 4 pairs sharing f's
        # squarings, as blst's multi-pairing does; kernels/k_mlq.hip); a chunk's
        # signature-sum pair runs the same loop
        ml = wm["ml_lines"] + mlf_products(wm, shape)
        ml1 = ml
        # the signature sums: one group sum over the pass and ONE signature Miller loop
        # (merged signature sum, $BLS_SIG_TOTAL), or one per chunk
        total = os.environ.get("BLS_SIG_TOTAL", "1") != "0" and chunks > 1
        msm = total and (bool(shape & 1) if shape is not None else os.environ.get("BLS_MSM", "0") == "1") \
            and "msm_madd" in wm
        r_sig = wm["chain_r_sig"]
        if msm:
            # kernels/k_msm.hip: 8 (window, digit) entries per set, one mixed addition each
            # (255 of 256 digits are non-zero), the mu image for the 4 b-half entries, a
            # bucket addition per segment, and per pass 4 windows x (256 x 8 + 255)
            # additions + 36 doublings + 3 additions
            seg = 8
            while seg * seg < (8 * n_sets + 1019) // 1020:
                seg *= 2
            fixed = (4 * (256 * 8 + 255) + 3) * wm["gsum_add"] + 36 * wm["g2_dbl"]
            r_sig = 0.0
            sums = (8 * 255 / 256 * wm["msm_madd"] + 4 * wm["msm_mu"] + 8 / seg * wm["gsum_add"] + fixed / n_sets
                    + (ml1 + wm["vset"]) / n_sets)
        elif total:
            sums = (ml1 + wm["vset"]) / n_sets + (n_sets - 1) / n_sets * wm["gsum_add"]
        else:
            sums = chunks / n_sets * (ml1 + wm["vset"]) + (n_sets - chunks) / n_sets * wm["gsum_add"]
        per = (wm["k_pre"] + wm["chain_h"] + wm["chain_subgroup"] + r_sig + wm["chain_r_pk"] + ml
               + sums + merged / n_sets)
        return per, ("k_pre %.0f + k_chain %.0f + k_mln %.0f + signature sums%s %.0f + merged check %.0f" %
                     (wm["k_pre"], wm["chain_h"] + wm["chain_subgroup"] + r_sig + wm["chain_r_pk"], ml,
                      " (Pippenger MSM + one ML)" if msm else "/ML", sums, merged / n_sets))
    S = pack_of(n_sets)
    ps = pset_products_per_set(S)
    return wm["k_pre"] + ps + merged / n_sets, "k_pre %.0f + k_pset %.0f + merged check %.0f" % (
        wm["k_pre"], ps, merged / n_sets)


def reference_work_per_set(reqs_per_chunk: int = 16, pairs_per_loop: int = 8) -> tuple[float, str]:
    """SURVEY §8d's reference-algorithm work W_set (blst-style verifyMultipleSignatures,
    no dedup, no units, no merged check): decompression + subgroup check, hash_to_G2,
    64-bit r sig and r pk, one Miller-loop pair per set with the squarings shared by
    `pairs_per_loop` pairs (blst's multi-pairing), and per chunk of `reqs_per_chunk`
    sets one signature pair and one final exponentiation.  Same stage counts as
    work_per_set (work_model.json, coop_programs.json)."""
    pg = json.loads((ROOT / "lodestar_amd" / "_native" / "coop_programs.json").read_text())
    wm = json.loads((ROOT / "lodestar_amd" / "_native" / "work_model.json").read_text())
    fe = pg["fin_fe1"]["mul_ops"] + pg["fin_fe2"]["mul_ops"]
    # f side per pair: 62 Fp12 squarings (36 products) shared, 68 sparse line products (39)
    f_pair = 62 * 36 / pairs_per_loop + 68 * 39
    per_set = (wm["k_pre"] + wm["chain_h"] + wm["chain_subgroup"] + wm["chain_r_sig"] + wm["chain_r_pk"]
               + wm["ml_lines"] + f_pair + wm["gsum_add"])
    per_chunk = wm["ml_lines"] + wm["ml_f_one"] + fe
    return per_set + per_chunk / reqs_per_chunk, (
        f"decompress + hash_to_G2 {wm['k_pre']:.0f} + cofactor {wm['chain_h']:.0f} + subgroup "
        f"{wm['chain_subgroup']:.0f} + r sig {wm['chain_r_sig']:.0f} + r pk {wm['chain_r_pk']:.0f} + Miller pair "
        f"{wm['ml_lines'] + f_pair:.0f} ({pairs_per_loop} pairs per loop) + sig sum {wm['gsum_add']:.0f} + per chunk of "
        f"{reqs_per_chunk} (signature pair + final exponentiation) {per_chunk:.0f}")


def latency_curve(ctxs, works, points, sets_per_call: int, steps: int = 5) -> dict:
    """sets/s and ms per call at (contexts, calls per pass) points below the headline's:
    the call latency a host gets for the rate it asks (each point one warm-up pass, then
    `steps` timed passes, verdicts checked)."""
    res = {}
    for c, k in points:
        if c > len(ctxs) or k > len(works[0][0]):
            continue
        batches = [w[0][:k] for w in works[:c]]
        timed_calls(ctxs[:c], batches, 1)
        el, _, ok = timed_calls(ctxs[:c], batches, steps)
        assert ok, f"latency curve {c}x{k}: verification failed"
        res[f"{c}x{k}"] = {"sets_in_flight": c * k * sets_per_call, "sets_per_s": round(c * k * sets_per_call * steps / el, 1),
                           "ms_per_call": round(el / steps * 1e3, 3)}
    return res


TIMED_SHAPE = "16 x 22"                    # the default timed region: contexts x calls per pass
PMC_FILE = "r06_pmc_timed_16x22.json"    # the committed counter summary the bench line cites (timed shape)
# the committed rocprofv3 --kernel-trace --stats summary of the timed 16 x 22 shape (the
# dominant kernels' average launch time with ~12 passes sharing the device)
KSTATS_FILE = "r06_kernel_stats_timed_16x22.csv"
KSTATS_SETS = 22528                      # sets per pass of that run (22 calls x 1024)
PEAK_FILE = "peak_fixed.json"            # the fixed v_mad_u64_u32 peak (median of the committed measurements)


def peak_fixed() -> float | None:
    p = ROOT / "profiles" / PEAK_FILE
    return json.loads(p.read_text())["peak_fixed_tmad_s"] if p.exists() else None


def committed_kernel_times(names=("k_mlf", "k_mlq", "k_chain", "k_pre")) -> dict:
    """Average launch ns per kernel (by plain name prefix) from the committed timed-shape
    kernel trace (profiles/KSTATS_FILE)."""
    import csv

    p = ROOT / "profiles" / KSTATS_FILE
    out = {}
    if not p.exists():
        return out
    for r in csv.DictReader(open(p)):
        n = r["Name"].replace("void ", "").split("(")[0]
        for k in names:
            if n.split("<")[0] == k:
                out[n] = float(r["AverageNs"])
    return out
VERIFY_KERNELS = ("k_pk", "k_pre", "k_chain", "k_gsum", "k_vset", "k_mlq", "k_mlf", "k_msm", "k_status", "k_fprod",
                  "k_chunk_coop", "k_indiv_coop", "k_fold", "k_exact", "k_uset", "k_gsum1", "k_mln")


def committed_pmc():
    """The SQ / HBM counters of one 32768-set pass (profiles/PMC_FILE: rocprofv3 --pmc
    passes over bench.py --probe-only, tools/pmc_summary.py), per verify kernel -- copied
    from the committed file, labelled as such; None if absent."""
    p = ROOT / "profiles" / PMC_FILE
    if not p.exists():
        return None
    d = json.loads(p.read_text())
    out, total, vset = {}, 0, 0.0
    sets = d.get("sets_per_pass")
    for name, v in d.get("kernels", {}).items():
        if not name.startswith(VERIFY_KERNELS):
            continue
        total += v.get("hbm_bytes_per_launch", 0)
        if sets and "SQ_INSTS_VALU" in v:
            vset += v["SQ_INSTS_VALU"] / sets  # per dispatch: every wave's VALU instructions
        wc = v.get("SQ_WAVE_CYCLES")
        if name.startswith(("k_chain", "k_mlf", "k_mlq", "k_pre")) and wc:
            out[name] = {"valu_issue_frac": round(v["SQ_ACTIVE_INST_VALU"] / wc, 3),
                         "waves_per_simd": v.get("waves_per_simd"), "valu_busy": v.get("valu_busy"),
                         "valu_insts_per_wave": round(v["SQ_INSTS_VALU"] / max(1.0, v["SQ_WAVES"])),
                         "valu_wave_insts_per_set": round(v["SQ_INSTS_VALU"] / sets) if sets else None,
                         "hbm_bytes_per_launch": v.get("hbm_bytes_per_launch")}
    # the timed shape proper (Pippenger signature sum, four items per k_mlf lane): counter
    # collection serialises the probe's kernels, so some passes start with fewer sets in
    # flight and take the group-sum shape (k_chain with role 2) or two items per k_mlf
    # lane; the timed shape is the one with the fewest instructions in both, so per kernel
    # the lowest per-dispatch figure
    per = d.get("per_dispatch_valu_wave_insts_per_set", {})
    mode = {n: min(v) for n, v in per.items() if v and n.startswith(VERIFY_KERNELS)}
    return {"source": f"profiles/{PMC_FILE} (copied, not measured by this run)", "shape": d.get("shape"),
            "kernels": out, "hbm_bytes_per_pass": total, "sets_per_pass": sets,
            "valu_wave_insts_per_set": round(vset) if sets else None,
            "valu_wave_insts_per_set_note": "average over every dispatch of the probe, mixed pass shapes",
            "valu_wave_insts_per_set_timed_shape": sum(mode.values()) if mode else None,
            "valu_wave_insts_per_set_timed_shape_by_kernel": mode or None}


def interop_sk(i: int) -> bytes:
    v = int.from_bytes(hashlib.sha256(i.to_bytes(32, "little")).digest(), "little") % R_ORDER
    return v.to_bytes(32, "big")


def make_workload(gpu, n_sets: int, rank: int, roots: int = 0):
    """cfg2: every set signs its own root.  roots > 0: the cfg5 mainnet-epoch shape
    (SURVEY §8d), consecutive sets in committees sharing `roots` signing roots per call.
    Returns (batch, call128, sets, raw96): the packed cfg2 call, a 128-set non-batchable
    call (cfg1 shape), the sets (table indices), the 96-byte uncompressed keys."""
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
    raw96, _ = gpu.aggregate_pubkeys([[j % n_keys] for j in range(n_sets)])
    batch = pack_requests([(True, [s]) for s in sets])
    call128 = pack_requests([(False, sets[:128])])
    return batch, call128, sets, raw96


# ---------------------------------------------------------------------------
# CPU baseline: the C++ restatement under oracle/cpu ("not blst"), host cores
# ---------------------------------------------------------------------------
def _cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or "unknown"


def _cpu_quota() -> float | None:
    """CPUs this process may use per the cgroup v2 quota (cpu.max), or None if unlimited."""
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        return None


def cpu_baseline(sets, raw96, threads: int | None = None, seconds: float = 10.0, latency_runs: int = 20) -> dict:
    """The reference's CPU path restated in C++ (oracle/cpu/bls_cpu.cpp): a worker pool
    of `threads` OS threads -- by default one per host core, the reference's pool size
    (os.cpus().length, multithread/poolSize.ts:3-11) -- each running
    verifyManySignatureSets on messages of 128 single-set batchable requests (the pool's
    MAX_SIGNATURE_SETS_PER_JOB = 128, index.ts:39; chunks of 16 requests,
    worker.ts:17,56) back to back for `seconds` -> cfg2 sets/s; and cfg1: one message
    holding one non-batchable request of 128 sets on one core, `latency_runs` runs ->
    p50 / p99 ms.  When a cgroup quota caps this process below the core count (the GPU
    box gives a 1-GPU job a share of the host), the pool still runs `threads` workers and
    the measured rate is what the quota allows; the one-core rate x cores is reported
    beside it as the whole-host figure."""
    threads = threads or os.cpu_count() or 1
    import ctypes

    from lodestar_amd._abi import BlsBatch
    from lodestar_amd.native import _ptr, pack_requests

    lib = ctypes.CDLL(str(ROOT / "oracle" / "cpu" / "libbls_cpu.so"))
    lib.cpu_pool_throughput.argtypes = [ctypes.POINTER(BlsBatch), ctypes.c_int, ctypes.c_double,
                                        ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint32)]
    lib.cpu_message_latency.argtypes = [ctypes.POINTER(BlsBatch), ctypes.c_int, ctypes.c_void_p]
    raw_sets = [(raw96[i], m, s) for i, (_, m, s) in enumerate(sets[:128])]

    def batch_of(pb):
        b = BlsBatch()
        b.n_sets, b.n_reqs = pb.n_sets, pb.n_reqs
        keep = []
        for f in ("req_set_offsets", "req_batchable", "messages", "signatures", "pubkeys", "set_pk_offsets",
                  "pk_indices", "signature_lens"):
            a = getattr(pb, f)
            keep.append(a)
            setattr(b, f, _ptr(a))
        return b, keep

    job, k1 = batch_of(pack_requests([(True, [s]) for s in raw_sets]))
    rate, msgs = ctypes.c_double(), ctypes.c_uint32()
    rc = lib.cpu_pool_throughput(ctypes.byref(job), threads, seconds, ctypes.byref(rate), ctypes.byref(msgs))
    assert rc == 0, "CPU baseline verification failed"
    call, k2 = batch_of(pack_requests([(False, raw_sets)]))
    ms = np.zeros(latency_runs, dtype=np.float64)
    assert lib.cpu_message_latency(ctypes.byref(call), latency_runs, _ptr(ms)) == 0
    # one worker alone: the per-core rate (a 1024-set message: 8 messages of 128)
    one, one_msgs = ctypes.c_double(), ctypes.c_uint32()
    assert lib.cpu_pool_throughput(ctypes.byref(job), 1, min(seconds, 5.0), ctypes.byref(one),
                                   ctypes.byref(one_msgs)) == 0
    quota = _cpu_quota()
    return {"value": round(rate.value, 1), "unit": "sets/s", "cores": threads, "kind": "port",
            "impl": "C++ restatement of the reference worker pool, not blst (oracle/cpu/bls_cpu.cpp: 6x64-bit "
                    "Montgomery words, portable __int128 code without blst's mulx/adx assembly, so slower per core "
                    "than Lodestar's workers; shared-squaring Miller loops, sum of r_i sig_i, one final exp per chunk)",
            "cpu": _cpu_model(), "nproc": os.cpu_count(),
            "cgroup_cpu_quota": quota,
            "per_core_sets_per_s": round(one.value, 1),
            "whole_host_sets_per_s_extrapolated": round(one.value * (os.cpu_count() or 1), 1),
            "whole_host_note": "EXTRAPOLATED, not measured: one worker's measured rate x nproc, the reference pool "
                               "on every core of this host with no quota (an upper bound: no memory-bandwidth or SMT "
                               "contention counted); `value` is what the pool measured under this job's quota",
            "sample": f"cfg2: {threads} worker threads (one per core, poolSize.ts:3-11) x messages of 128 batchable "
                      f"single-set requests for {seconds:.0f} s ({msgs.value} messages); one worker alone for "
                      f"{min(seconds, 5.0):.0f} s ({one_msgs.value} messages); cfg1: one 128-set non-batchable request "
                      f"on one core x {latency_runs}",
            "cfg1_p50_ms_128": round(float(np.percentile(ms, 50)), 2),
            "cfg1_p99_ms_128": round(float(np.percentile(ms, 99)), 2)}


# ---------------------------------------------------------------------------
# modes
# ---------------------------------------------------------------------------
def timed_calls(ctxs, batches, steps: int):
    """`steps` x len(ctxs) passes (a pass: one call, or a list of calls submitted together
    through bls_gpu_verify_many), all contexts starting at one barrier; each pass goes to
    whichever context is idle -- a shared count of the passes left, as the adapter hands
    queued jobs to an idle context (multithread/index.ts runJob) -- so a context the
    device happens to serve more slowly does fewer passes instead of holding the region
    open while the others idle (with a fixed `steps` each, the contexts' pass times spread
    84-97 ms at 16 x 22 and the region ended on the slowest, tools/pass_gap_probe.py).
    Context i runs its own calls batches[i].  Returns (elapsed s, mean stage_ms, all
    verdicts valid)."""
    n = len(ctxs)
    start = threading.Barrier(n + 1)
    stage_sum = np.zeros(8)
    ok = [True]
    shapes: dict[int, int] = {}
    lock = threading.Lock()
    left = [steps * n]

    def take() -> bool:
        with lock:
            if left[0] <= 0:
                return False
            left[0] -= 1
            return True

    def worker(i):
        start.wait()
        acc = np.zeros(8)
        good = True
        mine: dict[int, int] = {}
        while take():
            if isinstance(batches[i], list):
                vs, st = ctxs[i].verify_many(batches[i])
                good = good and all(bool((v == 1).all()) for v in vs)
            else:
                v, st = ctxs[i].verify_packed(batches[i])
                good = good and bool((v == 1).all())
            acc += np.array(st.stage_ms[:])
            mine[st.pass_shape] = mine.get(st.pass_shape, 0) + 1
        with lock:
            stage_sum[:] += acc
            ok[0] = ok[0] and good
            for k, c in mine.items():
                shapes[k] = shapes.get(k, 0) + c

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    timed_calls.shapes = shapes  # pass_shape -> passes, for the roofline's work pricing
    return time.perf_counter() - t0, stage_sum / max(1, steps * n), ok[0]


def run_calls(ctxs, packed, calls_per_pass: int):
    """Every call of `packed` once, `calls_per_pass` consecutive calls per
    bls_gpu_verify_many pass, each pass on whichever context is idle; all contexts start
    at one barrier.  Returns (elapsed s, verdict arrays in call order, summed stats dict)."""
    n = len(ctxs)
    start = threading.Barrier(n + 1)
    out = [None] * len(packed)
    tot = {"batch_retries": 0, "batch_sigs_success": 0, "merged_fail": 0, "passes": 0,
           # device time of the passes whose merged check failed / passed, and the failed
           # passes' per-stage times (bls_stats.stage_ms, summed; the chunk fallback is
           # device_ms minus the stages)
           "fail_device_ms": 0.0, "pass_device_ms": 0.0, "fail_stage_ms": np.zeros(8)}
    lock = threading.Lock()

    # passes of calls_per_pass consecutive calls, each to whichever context is idle (a
    # shared queue, as in timed_calls)
    groups = [list(range(g, min(g + calls_per_pass, len(packed)))) for g in range(0, len(packed), calls_per_pass)]
    nxt = [0]

    def worker(i):
        start.wait()
        while True:
            with lock:
                if nxt[0] >= len(groups):
                    return
                ks = groups[nxt[0]]
                nxt[0] += 1
            vs, st = ctxs[i].verify_many([packed[k] for k in ks])
            for k, v in zip(ks, vs):
                out[k] = v.copy()
            with lock:
                tot["batch_retries"] += st.batch_retries
                tot["batch_sigs_success"] += st.batch_sigs_success
                tot["merged_fail"] += 1 if st.merged_check == 2 else 0
                tot["merged_skipped"] = tot.get("merged_skipped", 0) + (1 if st.merged_check == 3 else 0)
                tot["passes"] += 1
                if st.merged_check in (2, 3):  # the chunks were checked one by one
                    tot["fail_device_ms"] += st.device_ms
                    tot["fail_stage_ms"] += np.array(st.stage_ms[:])
                else:
                    tot["pass_device_ms"] += st.device_ms

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    return time.perf_counter() - t0, out, tot


def steady_state(ctxs, w, pbs, calls_per_pass: int, jobs: int) -> dict:
    """The slice's job `jobs` times back to back in ONE timed region (every context keeps
    taking its next calls, no barrier between jobs), verdicts checked for every call:
    the steady-state rate beside the one-job figure (`sets_per_s`, which is close to one
    pass's latency when a job is a pass or two per context)."""
    from lodestar_amd import workloads as W

    el, out, _ = run_calls(ctxs, pbs * jobs, calls_per_pass)
    bad = [k for k in range(len(out)) if not W.verdicts_ok(w, k % len(pbs), out[k])]
    assert not bad, f"steady state: {len(bad)} calls with wrong verdicts (first {bad[0]})"
    return {"steady_jobs": jobs, "steady_elapsed_s": round(el, 4),
            "steady_sets_per_s": round(jobs * w.n_sets / el, 1),
            "steady_passes_per_context": round(len(out) / len(ctxs) / calls_per_pass, 1)}


def sub_records(n_keys: int, n_ctx: int, calls_per_pass: int, cfg4_sets: int, reps: int = 3,
                latency_runs: int = 10, cfg4_ctx: int = 4, cfg4_cpp: int = 32, cfg5_sets: int = 131_072,
                cfg5_roots: int = 256, jobs: int = 5, only: set | None = None) -> dict:
    """BASELINE configs 3 and 4 at N = 1: cfg3, one block-import call
    (latency, sets/s, pubkeys aggregated/s); cfg4 this GPU's slice of the 1M-set range-sync
    job (1/8: shard by call), once with range sync's own non-batchable 128-set calls and
    once with every set its own batchable request, so invalid sets fail the merged check
    and their chunks and the per-request fallback run (worker.ts:76-87).  Verdicts are
    checked against the sets' validity by construction (lodestar_amd/workloads.py)."""
    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    res = {}
    ctxs = [GpuContext(0) for _ in range(n_ctx)]
    try:
        t0 = time.perf_counter()
        W.load_table(ctxs, n_keys)
        res["table"] = {"keys": n_keys, "build_s": round(time.perf_counter() - t0, 2)}
        # cfg3: one block
        w3 = W.cfg3_block(ctxs[0], n_keys) if only is None or "cfg3" in only else None
        pb3 = W.packed_calls(w3)[0] if w3 is not None else None
        if w3 is not None:
            ctxs[0].verify_packed(pb3)  # warm-up
        lat, stage = [], np.zeros(8)
        for _ in range(latency_runs if w3 is not None else 0):
            t1 = time.perf_counter()
            v, st = ctxs[0].verify_packed(pb3)
            lat.append(time.perf_counter() - t1)
            stage += np.array(st.stage_ms[:])
            assert W.verdicts_ok(w3, 0, v), "cfg3 block call verdict wrong"
        if w3 is not None:
            p50 = statistics.median(lat)
            n3 = w3.n_sets
            keys3 = sum(len(s[0]) for s in w3.calls[0])
            res["cfg3"] = {"workload": w3.note, "sets": n3, "pubkeys": keys3, "p50_ms": round(p50 * 1e3, 3),
                           "p99_ms": round(float(np.percentile(np.array(lat) * 1e3, 99)), 3),
                           "sets_per_s": round(n3 / p50, 1), "pubkeys_aggregated_per_s": round(keys3 / p50, 1),
                           "stage_ms": {k: round(float(x) / latency_runs, 3) for k, x in zip(STAGE_NAMES, stage)}}
        # cfg4: this GPU's slice, both call shapes; calls of 128 sets, cfg4_cpp of them per
        # device pass on cfg4_ctx contexts (sets in flight = the product, stated)
        c4, cpp4 = ctxs[:cfg4_ctx], cfg4_cpp
        for key, batchable in (("cfg4_slice", False), ("cfg4_slice_batchable", True)):
            if only is not None and key not in only:
                continue
            w4 = W.cfg4_slice(ctxs[0], n_keys, cfg4_sets, batchable_calls=batchable)
            pbs = W.packed_calls(w4)
            run_calls(c4, pbs[: len(c4) * cpp4], cpp4)  # warm-up
            best, out, tot = None, None, None
            for _ in range(reps):
                el, out, tot = run_calls(c4, pbs, cpp4)
                best = el if best is None else min(best, el)
            bad = [k for k in range(len(pbs)) if not W.verdicts_ok(w4, k, out[k])]
            assert not bad, f"{key}: {len(bad)} calls with wrong verdicts (first {bad[0]})"
            n_inv = sum(not x for v in w4.valid for x in v)
            res[key] = {"workload": w4.note, "sets": w4.n_sets, "calls": len(pbs), "invalid_sets": n_inv,
                        "false_requests": sum(int((o == 0).sum()) for o in out),
                        "elapsed_s": round(best, 4), "sets_per_s": round(w4.n_sets / best, 1),
                        "contexts": len(c4), "calls_per_pass": cpp4, "sets_in_flight": len(c4) * cpp4 * 128,
                        "runs": reps,
                        "batch_retries": tot["batch_retries"], "batch_sigs_success": tot["batch_sigs_success"],
                        "passes_merged_check_failed": tot["merged_fail"],
                        "passes_merged_check_skipped": tot.get("merged_skipped", 0),
                        "verdicts": "every call matches the sets' validity by construction",
                        **steady_state(c4, w4, pbs, cpp4, jobs)}
        # cfg5: this GPU's slice of the mainnet epoch (1/8 of ~1M attestations over 2048
        # committee roots), calls of 1024 batchable single-set requests on the headline's
        # contexts, invalid sets included (their passes fail the merged check and run the
        # chunk and per-request fallback inside the timed region)
        # and the same epoch slice with every set valid (cfg5_slice_valid): the shape's own
        # rate -- with 1 invalid set in 2,048 about half of the 1024-set calls fail their
        # merged check and re-verify a chunk's 16 requests alone
        for key, n_invalid in (("cfg5_slice", max(1, cfg5_sets // 2048)), ("cfg5_slice_valid", 0)):
            if only is not None and key not in only:
                continue
            w5 = W.cfg5_slice(ctxs[0], n_keys, cfg5_sets, cfg5_roots, invalid=n_invalid)
            pbs = W.packed_calls(w5)
            cpp5 = (len(pbs) + n_ctx - 1) // n_ctx
            run_calls(ctxs, pbs[: n_ctx], 1)  # warm-up
            best, out, tot = None, None, None
            for _ in range(reps):
                el, out, tot = run_calls(ctxs, pbs, cpp5)
                best = el if best is None else min(best, el)
            bad = [k for k in range(len(pbs)) if not W.verdicts_ok(w5, k, out[k])]
            assert not bad, f"{key}: {len(bad)} calls with wrong verdicts (first {bad[0]})"
            res[key] = {"workload": w5.note, "sets": w5.n_sets, "calls": len(pbs),
                        "invalid_sets": sum(not x for v in w5.valid for x in v),
                        "false_requests": sum(int((o == 0).sum()) for o in out),
                        "elapsed_s": round(best, 4), "sets_per_s": round(w5.n_sets / best, 1),
                        "contexts": n_ctx, "calls_per_pass": cpp5, "runs": reps,
                        "batch_retries": tot["batch_retries"], "batch_sigs_success": tot["batch_sigs_success"],
                        "passes_merged_check_failed": tot["merged_fail"],
                        "passes_merged_check_skipped": tot.get("merged_skipped", 0),
                        "verdicts": "every call matches the sets' validity by construction",
                        **steady_state(ctxs, w5, pbs, cpp5, jobs)}
    finally:
        for c in ctxs:
            c.close()
    return res


def run_job_slice(ctxs, w, calls_per_pass: int, steps: int, warmup: int, dist=None) -> dict:
    """--mode cfg4 / cfg5 (shard by call): this rank's calls of the job
    (workloads.cfg4_slice / cfg5_slice with rank / world), `calls_per_pass` per
    bls_gpu_verify_many pass on every context; `steps` passes over the whole slice
    inside the timed region, verdicts checked against the sets' validity by
    construction after each.  Invalid sets run the merged-check failure and
    per-request fallback paths inside the region.  `ctxs` are GpuContexts on the box (any
    object with verify_many(list[PackedBatch]) -> (verdicts, stats) in the gloo dry
    run).  Returns elapsed (s, this rank), sets verified, stats totals."""
    from lodestar_amd import workloads as W

    pbs = W.packed_calls(w)
    for _ in range(warmup):
        run_calls(ctxs, pbs[: len(ctxs) * calls_per_pass], calls_per_pass)
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    tot = {"batch_retries": 0, "batch_sigs_success": 0, "merged_fail": 0, "passes": 0,
           # device time of the passes whose merged check failed / passed, and the failed
           # passes' per-stage times (bls_stats.stage_ms, summed; the chunk fallback is
           # device_ms minus the stages)
           "fail_device_ms": 0.0, "pass_device_ms": 0.0, "fail_stage_ms": np.zeros(8)}
    false_req = 0
    for _ in range(steps):
        _, out, st = run_calls(ctxs, pbs, calls_per_pass)
        bad = [k for k in range(len(pbs)) if not W.verdicts_ok(w, k, out[k])]
        assert not bad, f"{len(bad)} calls with wrong verdicts (first {bad[0]})"
        for k in tot:
            tot[k] += st[k]
        false_req += sum(int((o == 0).sum()) for o in out)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    tot["fail_stage_ms"] = [round(float(x), 3) for x in tot["fail_stage_ms"]]
    return {"elapsed_s": elapsed, "sets": w.n_sets * steps, "calls": len(pbs) * steps, "false_requests": false_req,
            **tot}


def expected_bad_shards(valid: list[bool], world: int) -> list[int]:
    """Ranks whose contiguous slice (shard.shard_bounds) of a sharded call holds an
    invalid set: what verify_call_sharded's localisation must report."""
    from lodestar_amd.shard import shard_bounds

    return [k for k, (b, e) in enumerate(shard_bounds(len(valid), world)) if not all(valid[b:e])]


def run_sharded_job(be, w, seed, steps, warmup, dist, device) -> dict:
    """--mode sharded --shape cfg4 / cfg5: every call of workload `w` (identical on every
    rank) is ONE call split over the ranks (verify_call_sharded): per-rank Fp12 partials,
    one all-gather of 588-byte records, one final exponentiation, and for a failing call
    the localisation (each rank's own final exponentiation + an all-gather of one byte),
    all inside the timed region.  The verdict and bad_shards of every call are checked
    against the sets' validity by construction."""
    from lodestar_amd.shard import verify_call_sharded

    world = dist.get_world_size() if dist is not None and dist.is_initialized() else 1

    def one_pass():
        for sets, valid in zip(w.calls, w.valid):
            ok, info = verify_call_sharded(sets, seed, be, dist, device, localize=True)
            assert ok is all(valid), f"sharded call verdict {ok}, expected {all(valid)}"
            assert info["bad_shards"] == expected_bad_shards(valid, world), info
    for _ in range(warmup):
        one_pass()
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        dist.barrier()
    return {"elapsed_s": elapsed, "sets": w.n_sets * steps, "calls": len(w.calls) * steps,
            "failing_calls": sum(not all(v) for v in w.valid) * steps}


def bench_job(args, ctxs, rank: int, world: int, dist, device, make_backend) -> dict:
    """--mode cfg4 / cfg5 (shard by call) and --mode sharded --shape cfg4 / cfg5 (each
    call split over the ranks).  The device pubkey table (args.table_keys interop keys)
    is loaded into every context first.  Returns rank 0's JSON record (value: all
    ranks' sets / the slowest rank's timed region)."""
    from lodestar_amd import workloads as W
    from lodestar_amd.shard import global_throughput

    W.load_table(ctxs, args.table_keys)
    if args.mode == "cfg4":
        w = W.cfg4_slice(ctxs[0], args.table_keys, args.cfg4_sets * world, rank=rank, world=world,
                         call_sets=args.cfg4_call_sets, agg_k=args.cfg4_agg_k, invalid_frac=args.cfg4_invalid)
        res = run_job_slice(ctxs, w, max(1, 4096 // args.cfg4_call_sets), args.steps, args.warmup, dist)
        workload = (f"cfg4 range-sync job of {args.cfg4_sets * world} sets sharded by call over {world} GPU(s) "
                    f"(this rank: {w.note})")
        par = f"shard-by-call x{world}"
    elif args.mode == "cfg5":
        w = W.cfg5_slice(ctxs[0], args.table_keys, args.cfg5_sets, args.cfg5_roots, call_sets=args.cfg5_call_sets,
                         invalid=max(1, args.cfg5_sets // 2048), rank=rank)
        res = run_job_slice(ctxs, w, 8, args.steps, args.warmup, dist)
        workload = f"cfg5 epoch slice per GPU, shard by call over {world} GPU(s) (this rank: {w.note})"
        par = f"shard-by-call x{world}"
    else:  # sharded
        n_call = args.sets * world
        if args.shape == "cfg4":
            w = W.cfg4_slice(ctxs[0], args.table_keys, 4 * n_call, call_sets=n_call, agg_k=args.cfg4_agg_k,
                             invalid_frac=args.cfg4_invalid / 50)
        else:
            w = W.cfg5_slice(ctxs[0], args.table_keys, 4 * n_call, 8, call_sets=n_call, invalid=2)
        seed = hashlib.sha256(b"sharded-job").digest()
        res = run_sharded_job(make_backend(ctxs[0]), w, seed, args.steps, args.warmup, dist, device)
        workload = (f"{args.shape} sharded calls: each of {len(w.calls)} calls of {n_call} sets split over {world} "
                    f"GPU(s) (per-rank Fp12 partial, 588-byte all-gather, one final exponentiation, bad-shard "
                    f"localisation of failing calls); {w.note}")
        par = f"sharded-call x{world}"
    value, elapsed = global_throughput(res["sets"] if args.mode != "sharded" else res["sets"] / world,
                                       res["elapsed_s"], dist, device=device)
    return {"metric": METRIC, "value": round(value, 2), "unit": "sets/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u32 (381-bit Fp, 12x32-bit Montgomery limbs)",
            "data": "synthetic: interop keys, sha256 messages, GPU-made signatures, invalid sets by construction",
            "config": {"workload": workload, "parallelism": par, "table_keys": args.table_keys,
                       "contexts_per_gpu": len(ctxs),
                       "runtime": {"hip_runtime": _mapped_hip(), "library_hip_runtime": _library_hip(),
                                   "process_group": ({"backend": dist.get_backend(), "world": dist.get_world_size()}
                                                     if dist is not None and dist.is_initialized() else None)}},
            "job": {k: v for k, v in res.items() if k != "elapsed_s"}}


def run_sharded(be, sets, seed, steps, warmup, dist, device):
    """--mode sharded: `steps` calls, each ONE call of every rank's sets (world x sets),
    verified as one random-scalar batch through verify_call_sharded with the partial
    backend `be` (GpuPartialBackend on the GPU box).  Returns (elapsed s, sets per call)."""
    from lodestar_amd.shard import verify_call_sharded

    for _ in range(warmup):
        ok, _ = verify_call_sharded(sets, seed, be, dist, device, localize=False)
        assert ok is True, "sharded warm-up call failed"
    if dist is not None:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        ok, _ = verify_call_sharded(sets, seed, be, dist, device, localize=False)
        assert ok is True, "sharded call failed inside the timed region"
    if dist is not None:
        dist.barrier()
    return time.perf_counter() - t0, len(sets)


def run_napi(work_file: Path, steps: int, inflight: int, n_sets: int, per_call: int = 1, max_call: int = 1024,
             devices: str = "0") -> dict:
    """--mode napi: integration/js/benchNapi.js in a child Node process (the GPU is not
    touched by this process meanwhile); per_call sets per verifySignatureSets call,
    max_call sets per GPU call (the adapter's maxSetsPerCall); `inflight` contexts per
    device slot of `devices` (the adapter's `devices` option)."""
    node = shutil.which("node")
    if node is None:
        raise SystemExit("--mode napi needs node")
    n_slots = len(devices.split(","))
    env = dict(os.environ, UV_THREADPOOL_SIZE=str(max(4, n_slots * inflight + 2)))
    out = subprocess.run([node, str(ROOT / "integration" / "js" / "benchNapi.js"), str(work_file), str(steps),
                          str(inflight), str(n_sets), str(per_call), str(max_call), devices], capture_output=True,
                         text=True, env=env, timeout=1200)
    if out.returncode != 0:
        raise SystemExit(f"benchNapi.js failed (exit {out.returncode}): {out.stderr[-2000:]} {out.stdout[-500:]}")
    return json.loads(out.stdout.strip().splitlines()[-1])


def _mapped_hip() -> list[str]:
    from lodestar_amd.native import mapped_hip_runtime

    return mapped_hip_runtime()


def _library_hip() -> str | None:
    """the libamdhip64 the library's HIP calls bind to (native.library_hip_runtime)"""
    from lodestar_amd.native import library_hip_runtime

    try:
        return library_hip_runtime()
    except Exception:  # noqa: BLE001 - a stand-in run without the library
        return None


def _free_port() -> int:
    import socket

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int, argv: list[str]) -> int:
    """`bench.py --gpus N` with no launcher around it (WORLD_SIZE unset): start N rank
    processes of this script, one per GPU (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    rendezvous on 127.0.0.1), before anything in this process touches a GPU -- the
    reference's pool splits the work across its workers the same way, one message per
    worker (multithread/index.ts:153-166).  Rank 0 prints the JSON line; a rank that
    fails stops the others; returns the worst exit status."""
    import threading

    port = _free_port()
    procs = []

    def forward(pipe):
        # rank 0's stdout: the JSON line to stdout, anything else a library printed there
        # (gloo's connection notes) to stderr, so stdout holds the one line
        for line in iter(pipe.readline, b""):
            (sys.stdout if line.lstrip().startswith(b"{") else sys.stderr).buffer.write(line)
            (sys.stdout if line.lstrip().startswith(b"{") else sys.stderr).flush()

    fwd = None
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, str(Path(__file__).resolve()), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else sys.stderr.fileno()))
        if r == 0:
            fwd = threading.Thread(target=forward, args=(procs[0].stdout,), daemon=True)
            fwd.start()
    worst = 0
    try:
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                worst = bad[0]
                for p in procs:
                    if p.poll() is None:
                        p.terminate()
                break
            time.sleep(0.2)
        for p in procs:
            try:
                p.wait(timeout=60)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        if fwd is not None:
            fwd.join(timeout=10)
    return worst or next((p.returncode for p in procs if p.returncode), 0)


def _stand_in(spec: str):
    """--stand-in MODULE:FACTORY: a CPU object answering the GpuContext calls the job
    modes make (tests/test_bench_jobs.py supplies one), so the rank launch and the
    job modes run without a device.  Test infrastructure only; never the measurement."""
    import importlib

    mod, _, name = spec.partition(":")
    return getattr(importlib.import_module(mod), name)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="GPUs of this node, one rank each: launched here when no launcher set WORLD_SIZE")
    ap.add_argument("--steps", type=int, default=16)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--sets", type=int, default=1024)
    ap.add_argument("--latency-runs", type=int, default=20)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--inflight", type=int, default=16, help="verifier contexts (HIP streams) per GPU")
    # default 16 contexts x 22 calls: the rate follows the sets in flight (profiles/r03_knee.json:
    # 4 x 16 2.29M at 29 ms per pass, 12 x 16 3.09M at 64 ms; past 200k sets in flight the
    # library switches to the Pippenger signature sum and four items per k_mlf lane).  Round 6
    # (profiles/r06_knee.json, alternated on one box): 12 x 22 3.51-3.56M at 76-77 ms, 16 x 16
    # 3.62-3.64M at 72 ms, 16 x 22 3.70-3.75M at 96-97 ms; 12 x 32 was faster still but past
    # 100 ms per pass.  A call's verdicts arrive when its pass ends, inside the reference's
    # 100 ms job buffering (multithread/index.ts:57 MAX_BUFFER_WAIT_MS).  16 contexts reserve
    # 16 x 322 MiB of scratch (k_chain), inside the library's 6 GiB admission budget (20 are
    # refused cleanly: BLS_ERR_ADMISSION; the runtime aborted queues past ~8 GiB,
    # profiles/r03_scratch_out_of_resources.txt)
    ap.add_argument("--calls-per-pass", type=int, default=22,
                    help="calls each context submits together per pass (bls_gpu_verify_many; each call keeps "
                         "its own chunks and verdicts)")
    ap.add_argument("--mode", choices=("cfg2", "sharded", "napi", "cfg4", "cfg5"), default="cfg2")
    ap.add_argument("--devices", default="0",
                    help="--mode napi: the JS adapter's device slots, comma-separated (one verifier per node; '0,0' "
                         "= two slots on one GPU); --inflight contexts are spread over them")
    ap.add_argument("--shape", choices=("cfg2", "cfg4", "cfg5"), default="cfg2",
                    help="--mode sharded: the sets of the split call (cfg2 all-valid single sets; cfg4 the range-sync "
                         "mix with aggregates and invalid sets; cfg5 committee-shared roots with invalid sets)")
    ap.add_argument("--cfg4-call-sets", type=int, default=128, help="sets per cfg4 call (range sync's batches)")
    ap.add_argument("--cfg4-agg-k", type=int, default=128, help="keys per cfg4 aggregate set")
    ap.add_argument("--cfg4-invalid", type=float, default=0.01, help="fraction of invalid cfg4 sets")
    ap.add_argument("--cfg5-sets", type=int, default=131_072, help="sets per GPU of --mode cfg5 (1M / 8)")
    ap.add_argument("--cfg5-call-sets", type=int, default=1024, help="sets per cfg5 call (gossip buffering)")
    ap.add_argument("--cfg5-roots", type=int, default=256, help="committee roots per GPU of --mode cfg5 (2048 / 8)")
    ap.add_argument("--roots", type=int, default=0,
                    help="distinct signing roots per call (0: all distinct, cfg2; 2: the cfg5 committee shape)")
    ap.add_argument("--no-dedup", action="store_true", help="hash every set's root (BLS_DEBUG_NO_MSG_DEDUP)")
    ap.add_argument("--no-units", action="store_true",
                    help="one Miller loop per set even for shared roots (BLS_DEBUG_NO_UNITS)")
    ap.add_argument("--no-sub-records", action="store_true", help="skip the cfg3 / cfg4 sub-records")
    ap.add_argument("--probe-only", action="store_true",
                    help="counter / trace runs: the warm-up and timed passes only (no latency, solo, peak or CPU "
                         "legs), so a profile holds exactly those launches")
    ap.add_argument("--table-keys", type=int, default=1 << 20, help="device pubkey table of the cfg3 / cfg4 records")
    ap.add_argument("--cfg4-sets", type=int, default=125_000,
                    help="sets of this GPU's cfg4 slice (1M sets over 8 GPUs by call)")
    # the cfg4 slice's knee: 8 x 64 in rounds 4-6 (profiles/r04_sweep_cfg4.json, one job: 12 x 64 left
    # contexts short of a second pass); with passes handed to idle contexts 12 x 64 leads in the steady
    # state (r06_sweep_cfg4.json: 2.56-2.62M / 1.89-1.92M vs 2.26-2.30M / 1.78-1.80M calls / per-set
    # requests; 16 x 64 2.72-2.78M / 1.61-1.64M)
    ap.add_argument("--cfg4-contexts", type=int, default=12,
                    help="contexts of the cfg4 sub-record (12 x 64: profiles/r06_sweep_cfg4.json)")
    ap.add_argument("--cfg4-calls-per-pass", type=int, default=64, help="128-set calls per pass of the cfg4 sub-record")
    ap.add_argument("--hw-queues", default="unset,4,16",
                    help="GPU_MAX_HW_QUEUES values of the deployable-configuration sub-records ('unset': the "
                         "variable removed; empty: none)")
    ap.add_argument("--no-merged-check", action="store_true",
                    help="one final exponentiation per chunk only (BLS_DEBUG_NO_MERGED_CHECK)")
    ap.add_argument("--hwq-child", action="store_true",
                    help="internal: the deployable-configuration sub-record (hw_queues_N), started by the parent "
                         "before it touches the GPU; waits for a line on stdin, then runs the cfg2 timed region")
    ap.add_argument("--torch-world1-child", action="store_true",
                    help="internal: the runtime_torch_world1 sub-record (torch.cuda.set_device + a world-1 nccl group "
                         "before the cfg2 timed region), started by the parent before it touches the GPU")
    ap.add_argument("--no-torch-world1", action="store_true", help="skip the runtime_torch_world1 sub-record")
    ap.add_argument("--stand-in", default=None, metavar="MODULE:FACTORY",
                    help="dry run of --mode cfg4 / cfg5 without a device: ranks on gloo, contexts from this CPU "
                         "stand-in (tests only)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        # one rank per GPU, launched before this process touches the GPU
        sys.exit(launch_ranks(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != max(1, args.gpus):
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: one rank per GPU")
    dist, device = None, None
    # $BLS_BENCH_SHARE_DEVICE=1: a rehearsal of the N-rank line on a box with fewer GPUs --
    # every rank on cuda:0, control collectives over gloo (the data path has none); the
    # line says so in `data`.  Not a measurement of N GPUs.
    share = os.environ.get("BLS_BENCH_SHARE_DEVICE") == "1" and world > 1
    if share:
        local_rank = 0
    if world > 1:
        # RCCL only where the path exchanges data: the split call (--mode sharded).  The
        # shard-by-request / by-call modes (cfg2, cfg4, cfg5) have no data-path collective;
        # their barrier and max-over-ranks reduction run on gloo, and the library is loaded
        # BEFORE torch so it binds to /opt/rocm's HIP runtime exactly as the N = 1 line does
        # (torch imported first would hand it torch's bundled libamdhip64 -- ROCm 7.0, the
        # same soname -- and the scaling curve would mix a runtime change into its N = 1 ->
        # N > 1 ratio; the line's config.runtime records which runtime ran, and the N = 1
        # line's runtime_torch_world1 sub-record measures the cfg2 shape under torch's).
        nccl = args.mode == "sharded" and not (args.stand_in or share)
        if not nccl and not args.stand_in:
            from lodestar_amd._abi import load_library

            load_library()
        import torch.distributed as dist

        if nccl:
            import torch

            torch.cuda.set_device(local_rank)
            device = f"cuda:{local_rank}"
            dist.init_process_group("nccl")
        else:
            dist.init_process_group("gloo")
    elif args.torch_world1_child:
        # the runtime_torch_world1 sub-record (started before the parent's first GPU call,
        # released after it): torch's HIP runtime and a world-1 RCCL group, as a rank of the
        # nccl modes has them, around the cfg2 timed region
        if sys.stdin.readline().strip() != "go":
            sys.exit(3)
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(0)
        device = "cuda:0"
        dist.init_process_group("nccl", rank=0, world_size=1)

    def barrier_sync():
        if dist is not None:
            dist.barrier()
            if device is not None:
                import torch

                torch.cuda.synchronize()

    if args.stand_in:
        if args.mode not in ("cfg4", "cfg5"):
            raise SystemExit("--stand-in runs the sharded-by-call job modes (cfg4, cfg5)")
        factory = _stand_in(args.stand_in)
        out = bench_job(args, [factory() for _ in range(args.inflight)], rank, world, dist, device, None)
        out["data"] += "; DRY RUN: CPU stand-in contexts (--stand-in), not a measurement"
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    # The deployable configuration (hw_queues_4 / hw_queues_16): the same cfg2 shape in
    # child processes whose HIP runtime gets GPU_MAX_HW_QUEUES = 4 (HIP's default, what a
    # beacon node that sets nothing runs) and 16, started now -- before this process makes
    # any GPU call -- and released one at a time after this process's own GPU work; each
    # times the parent's steps after the parent's warm-up (at least 2: the first passes
    # pick their shape from fewer sets in flight)
    hwq_children = {}
    if args.hwq_child:
        args.probe_only = True
        if sys.stdin.readline().strip() != "go":  # the parent's go: its own GPU work is done
            sys.exit(3)  # the parent ended without releasing this child: touch nothing
    elif args.torch_world1_child:
        args.probe_only = True
    elif (world == 1 and args.mode == "cfg2" and args.roots == 0 and not args.no_sub_records
          and not args.probe_only):
        if not args.no_torch_world1:
            env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
            env.pop("WORLD_SIZE", None)
            hwq_children["torch_world1"] = subprocess.Popen(
                [sys.executable, str(Path(__file__).resolve()), "--torch-world1-child", "--inflight",
                 str(args.inflight), "--calls-per-pass", str(args.calls_per_pass), "--steps",
                 str(args.steps), "--warmup", str(max(2, args.warmup)), "--sets", str(args.sets)],
                env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    if (world == 1 and args.mode == "cfg2" and args.roots == 0 and not args.no_sub_records and not args.probe_only
            and args.hw_queues and not args.hwq_child and not args.torch_world1_child):
        for q in args.hw_queues.split(","):
            env = {k: v for k, v in os.environ.items() if k != "GPU_MAX_HW_QUEUES"}
            if q != "unset":
                env["GPU_MAX_HW_QUEUES"] = str(int(q))
            hwq_children[q] = subprocess.Popen(
                [sys.executable, str(Path(__file__).resolve()), "--hwq-child", "--inflight", str(args.inflight),
                 "--calls-per-pass", str(args.calls_per_pass), "--steps", str(args.steps),
                 "--warmup", str(max(2, args.warmup)), "--sets", str(args.sets)],
                env=env, stdin=subprocess.PIPE, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True)
    try:
        _main_gpu(args, world, rank, local_rank, dist, device, share, barrier_sync, hwq_children)
    finally:
        for p in hwq_children.values():
            if p.poll() is None:
                p.kill()
                p.wait()


def run_hwq_children(children: dict, value: float | None = None) -> dict:
    """Release each deployable-configuration child in turn (this process's GPU work is
    over) and collect its line: sets/s and ms per call at its hardware-queue count, or
    under torch's HIP runtime with a world-1 RCCL group (runtime_torch_world1)."""
    res = {}
    for q, p in children.items():
        if q == "torch_world1":
            try:
                out, err = p.communicate("go\n", timeout=300)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
                res["runtime_torch_world1"] = {"error": "timed out"}
                continue
            lines = [ln for ln in out.splitlines() if ln.lstrip().startswith("{")]
            if p.returncode != 0 or not lines:
                res["runtime_torch_world1"] = {"error": f"exit {p.returncode}: {err[-400:]}"}
                continue
            d = json.loads(lines[-1])
            res["runtime_torch_world1"] = {
                "sets_per_s": d["value"], "ms_per_call": d["ms_per_step"], "steps": d["steps"],
                "contexts": d["config"]["contexts_per_gpu"], "calls_per_pass": d["config"]["calls_per_pass"],
                "runtime": d["config"].get("runtime"),
                "ratio_to_value": round(d["value"] / value, 4) if value else None,
                "note": "the headline's cfg2 shape in a child process that called torch.cuda.set_device(0) and "
                        "started a world-1 nccl (RCCL) group first, so the library runs on torch's bundled HIP "
                        "runtime, as a rank of the nccl modes does; the N > 1 cfg2 / cfg4 / cfg5 ranks instead "
                        "load the library before torch and use gloo for their barrier (no data-path collective), "
                        "so they run on the same runtime as the headline"}
            continue
        try:
            out, err = p.communicate("go\n", timeout=300)
        except subprocess.TimeoutExpired:
            p.kill()
            p.wait()
            res[f"hw_queues_{q}"] = {"error": "timed out"}
            continue
        lines = [ln for ln in out.splitlines() if ln.lstrip().startswith("{")]
        if p.returncode != 0 or not lines:
            res[f"hw_queues_{q}"] = {"error": f"exit {p.returncode}: {err[-400:]}"}
            continue
        d = json.loads(lines[-1])
        res[f"hw_queues_{q}"] = {
            "GPU_MAX_HW_QUEUES": q, "sets_per_s": d["value"], "ms_per_call": d["ms_per_step"],
            "contexts": d["config"]["contexts_per_gpu"], "calls_per_pass": d["config"]["calls_per_pass"],
            "steps": d["steps"],
            "note": "the headline's cfg2 shape in a child process started before the parent's first GPU call, " + (
                "GPU_MAX_HW_QUEUES unset: what a host that configures nothing runs (the Python wrapper asks for 24 "
                "queues as it loads the library, lodestar_amd/_abi.py, as the JS adapter does; the library itself "
                "never writes the environment)" if q == "unset" else
                f"its HIP runtime given GPU_MAX_HW_QUEUES={q} explicitly" + (" (HIP's own default)" if q == "4" else ""))
                    + "; the headline line runs with 24 (one hardware queue per context)"}
    return res


def _main_gpu(args, world, rank, local_rank, dist, device, share, barrier_sync, hwq_children) -> None:
    from lodestar_amd._abi import DEBUG_NO_MERGED_CHECK, DEBUG_NO_MSG_DEDUP, DEBUG_NO_UNITS
    from lodestar_amd.native import GpuContext
    from lodestar_amd.shard import GpuPartialBackend, global_throughput

    if args.mode in ("cfg4", "cfg5") or (args.mode == "sharded" and args.shape != "cfg2"):
        ctxs = [GpuContext(local_rank) for _ in range(args.inflight if args.mode != "sharded" else 1)]
        try:
            out = bench_job(args, ctxs, rank, world, dist, device,
                            lambda c: GpuPartialBackend(c))
        finally:
            for c in ctxs:
                c.close()
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return

    flags =((DEBUG_NO_MSG_DEDUP if args.no_dedup else 0) | (DEBUG_NO_MERGED_CHECK if args.no_merged_check else 0)
             | (DEBUG_NO_UNITS if args.no_units else 0))
    inflight = args.inflight if args.mode == "cfg2" else 1
    ctxs = [GpuContext(local_rank) for _ in range(inflight)]
    gpu = ctxs[0]
    K = max(1, args.calls_per_pass) if args.mode in ("cfg2", "napi") else 1
    works = [make_workload(c, args.sets * K, rank, args.roots) for c in ctxs]
    all_sets = works[0][2]  # every distinct set of context 0 (the N-API work file)
    if K > 1:
        from lodestar_amd.native import pack_requests as _pack

        # K calls of args.sets distinct sets per context (distinct signing roots, so no
        # cross-call dedup), each its own message
        works = [([_pack([(True, [s]) for s in w[2][k * args.sets:(k + 1) * args.sets]]) for k in range(K)],
                  _pack([(False, w[2][:128])]), w[2][:args.sets], w[3][:args.sets]) for w in works]
    for c in ctxs:
        c.set_debug_flags(flags)
    batch, call128, sets, raw96 = works[0]
    if isinstance(batch, list):
        batch = batch[0]  # one call of the pass: the solo-launch roofline probe below
    S = pack_of(args.sets)
    extra = {}

    if args.mode == "cfg2":
        for c, w in zip(ctxs, works):
            for _ in range(args.warmup):
                vs = c.verify_many(w[0])[0] if K > 1 else [c.verify_packed(w[0])[0]]
                assert all((v == 1).all() for v in vs), "warm-up verification failed"
        barrier_sync()
        elapsed, stage_ms, ok = timed_calls(ctxs, [w[0] for w in works], args.steps)
        barrier_sync()
        if not ok:
            raise SystemExit("verification failed inside the timed region")
        local_sets = args.sets * K * args.steps * inflight
        value, elapsed = global_throughput(local_sets, elapsed, dist, device=device)
        workload = ("cfg2: 1024 single-pubkey gossip sets per call, batchable requests, random-scalar batch in "
                    "chunks of 16 requests" if args.roots == 0 else
                    f"cfg5 shape: {args.sets} single-pubkey sets per call over {args.roots} committee-shared signing "
                    "roots, batchable requests" + (", root dedup off" if args.no_dedup else ""))
        workload += ", merged check off" if args.no_merged_check else ""
        workload += ", one Miller loop per set" if args.no_units else ""
        if K > 1:
            workload += (f"; each of the {inflight} contexts submits {K} calls per pass (bls_gpu_verify_many, "
                         "one device pass, chunks and verdicts per call)")
        config = {"workload": workload, "sets_per_call": args.sets, "contexts_per_gpu": inflight,
                  "calls_per_pass": K, "calls_in_flight_per_gpu": inflight * K,
                  "sets_per_step_per_gpu": args.sets * K * inflight, "parallelism": f"shard-by-request x{world}",
                  "call_latency_ms": round(elapsed / max(1, args.steps) * 1e3, 3)}
        scaling = "weak"
    elif args.mode == "sharded":
        # the call: every rank's sets (each rank made its own keys/messages; the call's
        # pubkeys travel raw, as the worker wire format, index.ts:160)
        mine = [(raw96[i], m, s) for i, (_, m, s) in enumerate(sets)]
        all_sets = mine
        if dist is not None:
            gathered = [None] * world
            dist.all_gather_object(gathered, mine)
            all_sets = [s for part in gathered for s in part]
        seed = hashlib.sha256(b"sharded-bench").digest()
        from lodestar_amd.shard import GpuPartialBackend

        elapsed_local, total = run_sharded(GpuPartialBackend(gpu), all_sets, seed, args.steps, args.warmup, dist,
                                           device)
        value, elapsed = global_throughput(total * args.steps / world, elapsed_local, dist, device=device)
        stage_ms = np.zeros(8)
        config = {"workload": f"cfg4/cfg5 sharded call: one call of {total} single-pubkey sets split over {world} "
                              "GPU(s); per-rank Fp12 Miller-loop partial, all-gather of 588-byte records, one final "
                              "exponentiation", "sets_per_call": total, "sets_per_step_per_gpu": args.sets,
                  "parallelism": f"sharded-call x{world}"}
        scaling = "weak"
    else:  # napi
        if world > 1:
            raise SystemExit("--mode napi runs on one GPU")
        with tempfile.TemporaryDirectory() as td:
            # sets * calls_per_pass distinct sets: a GPU call of max_call sets holds no
            # repeated signing root (no dedup advantage over the cfg2 line)
            sets = all_sets
            pks48 = gpu.sk_to_pk(b"".join(interop_sk(i) for i in range(len(sets)))).tobytes()
            wf = Path(td) / "work.json"
            wf.write_text(json.dumps({"pubkeys48": pks48.hex(),
                                      "sets": [{"idx": pk[0], "msg": m.hex(), "sig": s.hex()} for pk, m, s in sets]}))
            for c in ctxs:
                c.close()
            ctxs = []
            max_call = len(sets)
            slots = len(args.devices.split(","))
            per_slot = max(1, args.inflight // slots)  # the same contexts in total, spread over the slots
            batched = run_napi(wf, args.steps, per_slot, len(sets), args.sets, max_call, args.devices)
            res = run_napi(wf, args.steps, per_slot, len(sets), 1, max_call, args.devices)
        value, elapsed = res["sets_per_s"], res["elapsed_s"]
        stage_ms = np.zeros(8)
        extra["napi"] = {"per_set_calls": res, "calls_of_1024_sets": batched,
                         "note": "per-set calls: one JS promise per attestation, bound by the Node main thread; "
                                 "calls of 1024 sets (sync / block-import shape): bound by the GPU"}
        config = {"workload": "cfg2 through the N-API addon + JS GpuBlsVerifier: one verifySignatureSets([set], "
                              f"{{batchable: true}}) per set, buffered and coalesced into GPU calls of up to {max_call} "
                              "sets", "sets_per_step_per_gpu": res.get("sets_per_step"), "contexts": args.inflight,
                  "devices": args.devices, "contexts_per_slot": per_slot,
                  "parallelism": f"napi x1 ({slots} device slot(s): {args.devices})"}
        scaling = "weak"

    from lodestar_amd.native import mapped_hip_runtime

    # which HIP runtime the library runs under (torch's bundled copy once a rank has
    # initialised torch.cuda / RCCL, /opt/rocm's otherwise) and the process group
    config["runtime"] = {"hip_runtime": mapped_hip_runtime(), "library_hip_runtime": _library_hip(),
                         "process_group": ({"backend": dist.get_backend(), "world": dist.get_world_size()}
                                           if dist is not None and dist.is_initialized() else None)}
    out = None
    if rank == 0:
        out = {"metric": METRIC, "value": round(value, 2), "unit": "sets/s", "n_gpus": world, "steps": args.steps,
               "warmup": args.warmup, "ms_per_step": round(elapsed / max(1, args.steps) * 1e3, 3),
               "higher_is_better": True, "scaling": scaling, "vs_baseline": None,
               "dtype": "u32 (381-bit Fp, 12x32-bit Montgomery limbs)",
               "data": "synthetic: interop keys, sha256 messages, GPU-made signatures", "config": config}
        if share:
            out["data"] += f"; REHEARSAL: {world} ranks sharing one GPU (BLS_BENCH_SHARE_DEVICE), not an N-GPU figure"
        out.update(extra)

    if args.probe_only:
        for c in ctxs:
            c.close()
        if rank == 0:
            print(json.dumps(out), flush=True)
        if dist is not None:
            dist.destroy_process_group()
        return
    if args.mode != "napi":
        # p50 latency of one 128-set non-batchable call (cfg1 shape)
        lat = []
        for _ in range(args.latency_runs):
            t1 = time.perf_counter()
            v, _ = gpu.verify_packed(call128)
            lat.append((time.perf_counter() - t1) * 1e3)
            assert v[0] == 1
        # Roofline (VALU integer multiply-add bound; unit = v_mad_u64_u32, peak measured by
        # bls_gpu_mad_peak).  Algorithmic work = Fp Montgomery products x 288 MADs, per set
        # and per kernel from work_model.json / coop_programs.json (work_per_set).
        #   achieved / frac: the device-wide useful MAD rate over the timed region (every
        #     kernel of the pass; the contexts' launches overlap, so this is the figure that
        #     says how much of the chip the pipeline uses);
        #   kernels: per dominant kernel, its algorithmic MADs per launch / its average launch
        #     time from HIP events on its context's stream (stage_ms: in the timed region,
        #     where ~contexts launches share the device, and in solo passes of the same
        #     K calls with the device to itself).
        shapes = getattr(timed_calls, "shapes", {}) if args.mode == "cfg2" else {}
        shape = max(shapes, key=shapes.get) if shapes else None  # the timed passes' usual shape
        fpm_set, fpm_note = work_per_set(args.sets * K, shape=shape)  # one device pass: K calls
        mad_set = fpm_set * MADS_PER_FPM
        agg = (shape != 0) if shape is not None else sigagg_of(args.sets * K, inflight * args.sets * K)
        solo_st = []
        for _ in range(3):
            if K > 1:
                _, st = gpu.verify_many(works[0][0])
            else:
                _, st = gpu.verify_packed(batch)
            solo_st.append(np.array(st.stage_ms[:]))
            solo_shape = st.pass_shape
        solo_stage = np.median(np.array(solo_st), axis=0)
        peak_rate, _ = gpu.mad_peak()
        peak = peak_rate / 1e12
        per_gpu = value / world
        achieved = per_gpu * mad_set / 1e12
        if rank == 0:
            wm = json.loads((ROOT / "lodestar_amd" / "_native" / "work_model.json").read_text())
            pass_sets = args.sets * K
            kern = {}
            if agg:
                def per_kernel(sh):  # Fp products per set of k_chain and the Miller loops
                    msm = bool(sh & 1) if sh is not None else os.environ.get("BLS_MSM", "0") == "1"
                    return {"k_chain": wm["chain_h"] + wm["chain_subgroup"] + wm["chain_r_pk"]
                            + (0.0 if msm else wm["chain_r_sig"]),
                            "miller_loops": wm["ml_lines"] + mlf_products(wm, sh)}

                pk_timed, pk_solo = per_kernel(shape), per_kernel(solo_shape)
                for name, fpm in pk_timed.items():
                    if fpm is None:
                        continue
                    i = STAGE_NAMES.index(name)
                    mads, mads_solo = pass_sets * fpm * MADS_PER_FPM, pass_sets * pk_solo[name] * MADS_PER_FPM
                    t_timed, t_solo = float(stage_ms[i]), float(solo_stage[i])
                    kern[name] = {
                        "mad_per_launch": round(mads),
                        "fp_products_per_set": round(fpm, 1),
                        "fp_products_per_set_solo": round(pk_solo[name], 1),
                        "launch_ms_timed": round(t_timed, 3), "launch_ms_solo": round(t_solo, 3),
                        "achieved_timed": round(mads / (t_timed * 1e-3) / 1e12, 4) if t_timed > 0 else None,
                        "achieved_solo": round(mads_solo / (t_solo * 1e-3) / 1e12, 4) if t_solo > 0 else None,
                        "frac_solo": round(mads_solo / (t_solo * 1e-3) / 1e12 / peak, 4) if t_solo > 0 else None}
            if shapes:
                extra_shape = {str(k): v for k, v in sorted(shapes.items())}
                out["pass_shape"] = {"timed": extra_shape, "solo": solo_shape,
                                     "note": "bls_stats.pass_shape -> passes: bit 0 Pippenger signature sum, "
                                             "bits 8-15 items per k_mlf lane (both chosen by the sets in flight)"}
            pf = peak_fixed()
            if agg:
                # the dominant kernel in the timed shape (k_mlf, one lane per 1 / 2 / 4 items), from the
                # committed trace of that shape: algorithmic MADs per launch / its average launch time
                times = committed_kernel_times()
                for name, ns in times.items():
                    base = name.split("<")[0]
                    fpm = {"k_mlf": mlf_products(wm, 0x401), "k_mlq": wm["ml_lines"],
                           "k_chain": wm["chain_h"] + wm["chain_subgroup"] + wm["chain_r_pk"],
                           "k_pre": wm["k_pre"]}[base]
                    mads = KSTATS_SETS * fpm * MADS_PER_FPM
                    kern.setdefault(name, {}).update({
                        "mad_per_launch_timed_shape": round(mads), "fp_products_per_set": round(fpm, 1),
                        "launch_ms_timed_committed": round(ns / 1e6, 3),
                        "achieved_timed": round(mads / (ns * 1e-9) / 1e12, 4),
                        "frac_timed": round(mads / (ns * 1e-9) / 1e12 / pf, 4) if pf else None,
                        "source": f"profiles/{KSTATS_FILE} (copied: rocprofv3 kernel trace of the timed {TIMED_SHAPE} "
                                  f"shape, {KSTATS_SETS} sets per launch, four items per k_mlf lane; frac against "
                                  "peak_fixed)"})
            for v in kern.values():
                if pf and v.get("achieved_solo") is not None:
                    v["frac_solo_fixed"] = round(v["achieved_solo"] / pf, 4)
            roof = {"bound": "valu",
                    "kernel": ("every kernel of the pass; dominant: k_chain (per-set scalar chains) and the split "
                               "SIMT Miller loops (k_mlq + k_mlf)") if agg else "k_pset",
                    "achieved": round(achieved, 4),
                    "peak": round(peak, 3), "unit": "TMAD/s (v_mad_u64_u32)", "frac": round(achieved / peak, 5),
                    "peak_fixed": pf, "frac_fixed": round(achieved / pf, 5) if pf else None,
                    "peak_fixed_note": f"profiles/{PEAK_FILE}: median of every committed bls_gpu_mad_peak measurement; "
                                       "`frac_fixed` compares across boxes, `frac` uses this box's own measured peak",
                    "traffic": None,
                    "work": f"{fpm_set:.0f} Fp products/set ({fpm_note}) x {MADS_PER_FPM} MAD x "
                            f"{per_gpu:.0f} sets/s per GPU over the timed region",
                    "kernels": kern,
                    "peak_note": "measured: bls_gpu_mad_peak, every CU at 8 waves/SIMD"}
            pmc = committed_pmc()
            if pmc:
                roof["pmc"] = pmc
                roof["traffic"] = pmc["hbm_bytes_per_pass"]
                roof["traffic_note"] = ("HBM bytes (FETCH_SIZE x 2 + WRITE_SIZE, MI355X_MICROARCH.md) summed over every "
                                        "verify kernel of one pass of the committed counter run, NOT measured by this "
                                        f"run: {pmc['source']}")
            w_ref, w_ref_note = reference_work_per_set()
            roof["reference_equivalent"] = {
                "fp_products_per_set": round(w_ref), "work": w_ref_note,
                "achieved": round(per_gpu * w_ref * MADS_PER_FPM / 1e12, 4),
                "frac": round(per_gpu * w_ref * MADS_PER_FPM / 1e12 / peak, 5),
                "frac_fixed": round(per_gpu * w_ref * MADS_PER_FPM / 1e12 / pf, 5) if pf else None,
                "note": "SURVEY 8d: the reference algorithm's Fp products per set (blst-style, no dedup / units / "
                        "merged check) at this line's rate -- the work the reference would do for the same sets; "
                        "`frac` above prices the products this build executes"}
            out["p50_latency_ms_128"] = round(statistics.median(lat), 3)
            out["stage_ms"] = {k: round(float(x), 3) for k, x in zip(STAGE_NAMES, stage_ms)}
            out["roofline"] = roof
            if world == 1 and not args.no_cpu_baseline and args.mode == "cfg2":
                out["cpu_baseline"] = cpu_baseline(sets, raw96, seconds=args.cpu_seconds,
                                                   latency_runs=args.latency_runs)
                out["cpu_baseline"]["gpu_over_measured_pool"] = round(value / max(1e-9, out["cpu_baseline"]["value"]), 2)
                out["cpu_baseline"]["gpu_over_whole_host_extrapolated"] = round(
                    value / max(1e-9, out["cpu_baseline"]["whole_host_sets_per_s_extrapolated"]), 2)
    if world == 1 and args.mode == "cfg2" and args.roots == 0 and not args.no_sub_records and K > 1:
        curve = latency_curve(ctxs, works, ((4, 1), (8, 1), (4, 16), (8, 16)), args.sets)
        curve[f"{inflight}x{K}"] = {"sets_in_flight": inflight * K * args.sets, "sets_per_s": round(value, 1),
                                    "ms_per_call": out["ms_per_step"], "note": "the headline line"}
        out["latency_curve"] = curve
    for c in ctxs:
        c.close()
    ctxs = []
    if world == 1 and args.mode == "cfg2" and args.roots == 0 and not args.no_sub_records:
        out.update(sub_records(args.table_keys, inflight, K, args.cfg4_sets, cfg4_ctx=args.cfg4_contexts,
                               cfg4_cpp=args.cfg4_calls_per_pass, cfg5_sets=args.cfg5_sets,
                               cfg5_roots=args.cfg5_roots))
    if hwq_children:
        out.update(run_hwq_children(hwq_children, value))
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
