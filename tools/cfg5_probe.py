"""The cfg5 per-GPU slice (bench.py sub-record cfg5_slice) with and without its invalid
sets, `--jobs` jobs back to back each after a warm-up (the steady state of bench.py's
sub-record), for a kernel trace of where the failing passes
spend their time.  Prints one JSON object: per run the elapsed time, sets/s, passes
whose merged check failed, and the summed per-stage device times of the passes
(bls_stats.stage_ms: h2d, pk, pre, chain, sums, Miller loops, status + chunk fallback,
individual requests).

  python tools/cfg5_probe.py [--contexts 12] [--sets 131072] [--roots 256] [--invalid 64] [--runs invalid,valid]
"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
# the hardware queues of bench.py's timed region (12 contexts on HIP's default 4 queues
# serialise; set before anything starts the HIP runtime)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4") or 4) < 24:
    os.environ["GPU_MAX_HW_QUEUES"] = "24"


def run(ctxs, pbs, cpp):
    n = len(ctxs)
    start = threading.Barrier(n + 1)
    stage = np.zeros(8)
    tot = {"passes": 0, "merged_fail": 0, "batch_retries": 0, "device_ms": 0.0}
    lock = threading.Lock()
    out = [None] * len(pbs)

    def worker(i):
        mine = list(range(i, len(pbs), n))
        start.wait()
        for g in range(0, len(mine), cpp):
            ks = mine[g:g + cpp]
            vs, st = ctxs[i].verify_many([pbs[k] for k in ks])
            for k, v in zip(ks, vs):
                out[k] = v.copy()
            with lock:
                tot["passes"] += 1
                tot["merged_fail"] += 1 if st.merged_check == 2 else 0
                tot["batch_retries"] += st.batch_retries
                tot["device_ms"] += st.device_ms
                stage[:] += np.array(st.stage_ms[:])

    th = [threading.Thread(target=worker, args=(i,)) for i in range(n)]
    for t in th:
        t.start()
    start.wait()
    t0 = time.perf_counter()
    for t in th:
        t.join()
    return time.perf_counter() - t0, out, tot, stage


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contexts", type=int, default=12)
    ap.add_argument("--sets", type=int, default=131_072)
    ap.add_argument("--roots", type=int, default=256)
    ap.add_argument("--invalid", type=int, default=64)
    ap.add_argument("--table-keys", type=int, default=1 << 20)
    ap.add_argument("--runs", default="invalid,valid", help="which of the two jobs to run")
    ap.add_argument("--jobs", type=int, default=5, help="the job back to back in one timed region (steady state)")
    ap.add_argument("--shape", choices=("cfg5", "cfg4", "cfg4b"), default="cfg5",
                    help="cfg4 / cfg4b: bench.py's cfg4 slice (125,000 range-sync sets, 1 %% invalid) as "
                         "non-batchable or per-set batchable 128-set calls; --contexts / --cpp as its sub-record")
    ap.add_argument("--cpp", type=int, default=0, help="calls per pass (0: the slice's calls over the contexts)")
    args = ap.parse_args()
    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    ctxs = [GpuContext(0) for _ in range(args.contexts)]
    res = {"contexts": args.contexts, "stage_names": ["h2d", "k_pk", "k_pre", "k_chain", "sig_sums",
                                                       "miller_loops", "k_status+k_chunk", "k_indiv"]}
    try:
        W.load_table(ctxs, args.table_keys)
        for key, inv in (("invalid", args.invalid), ("valid", 0)):
            if key not in args.runs.split(","):
                continue
            if args.shape == "cfg5":
                w = W.cfg5_slice(ctxs[0], args.table_keys, args.sets, args.roots, invalid=inv)
            else:
                w = W.cfg4_slice(ctxs[0], args.table_keys, args.sets, invalid_frac=0.01 if inv else 0.0,
                                 batchable_calls=args.shape == "cfg4b")
            pbs = W.packed_calls(w)
            cpp = args.cpp or (len(pbs) + len(ctxs) - 1) // len(ctxs)
            run(ctxs, pbs[:len(ctxs)], 1)  # warm-up
            el, out, tot, stage = run(ctxs, pbs * args.jobs, cpp)
            bad = [k for k in range(len(out)) if not W.verdicts_ok(w, k % len(pbs), out[k])]
            assert not bad, f"{key}: {len(bad)} calls with wrong verdicts"
            res[key] = {"shape": args.shape, "invalid_sets": sum(not x for v in w.valid for x in v), "calls": len(pbs), "calls_per_pass": cpp, "elapsed_s": round(el, 4),
                        "jobs": args.jobs, "sets_per_s": round(args.jobs * w.n_sets / el, 1), **tot,
                        "stage_ms_sum": [round(float(x), 2) for x in stage]}
            print(key, json.dumps(res[key]), file=sys.stderr, flush=True)
    finally:
        for c in ctxs:
            c.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
