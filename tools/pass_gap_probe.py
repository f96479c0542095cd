"""Where a cfg2 pass's wall time goes outside its device stages, at the timed region's
shape (16 contexts x 22 calls): per pass, the library call's duration against its
device time (bls_stats.device_ms: first to last event on the stream) and the gap between
a context's consecutive calls (the harness's Python side).  Measurement tool.

  python tools/pass_gap_probe.py [--inflight 16] [--calls-per-pass 22] [--steps 6]"""
import argparse
import json
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--inflight", type=int, default=16)
    ap.add_argument("--calls-per-pass", type=int, default=22)
    ap.add_argument("--steps", type=int, default=6)
    a = ap.parse_args()
    from lodestar_amd.native import GpuContext, pack_requests

    ctxs = [GpuContext(0) for _ in range(a.inflight)]
    try:
        n = 1024 * a.calls_per_pass
        # the bench's own cfg2 work (bench.make_workload), split into 1024-set calls
        w = bench.make_workload(ctxs[0], n, 0, 0)
        sets = w[2]
        pks48 = ctxs[0].sk_to_pk(b"".join(bench.interop_sk(i) for i in range(len(sets)))).tobytes()
        for c in ctxs[1:]:
            c.load_pubkeys(pks48, 48)
        calls = [pack_requests([(True, [s]) for s in sets[k:k + 1024]]) for k in range(0, len(sets), 1024)]
        rec = [[] for _ in ctxs]
        start = threading.Barrier(len(ctxs) + 1)

        tot = [0.0] * len(ctxs)

        def worker(i):
            start.wait()
            t_prev = None
            t_first = None
            for s in range(a.steps + 2):
                t0 = time.perf_counter()
                vs, st = ctxs[i].verify_many(calls)
                t1 = time.perf_counter()
                if s >= 2:
                    if t_first is None:
                        t_first = t0
                    rec[i].append({"call_ms": (t1 - t0) * 1e3, "device_ms": st.device_ms,
                                   "gap_ms": (t0 - t_prev) * 1e3 if t_prev else 0.0})
                t_prev = t1
            tot[i] = t_prev - t_first

        th = [threading.Thread(target=worker, args=(i,)) for i in range(len(ctxs))]
        for t in th:
            t.start()
        start.wait()
        for t in th:
            t.join()
        allr = [r for rs in rec for r in rs]
        out = {k: round(float(np.mean([r[k] for r in allr])), 3) for k in ("call_ms", "device_ms", "gap_ms")}
        out["host_in_call_ms"] = round(out["call_ms"] - out["device_ms"], 3)
        out["passes"] = len(allr)
        per_ctx = [float(np.mean([r["call_ms"] for r in rs])) for rs in rec]
        out["call_ms_per_context_min_max"] = [round(min(per_ctx), 3), round(max(per_ctx), 3)]
        # the bench's definition: every context's sets over the slowest context's time
        out["sets_per_s_slowest"] = round(len(ctxs) * a.steps * n / max(tot), 1)
        out["sets_per_s_mean"] = round(len(ctxs) * a.steps * n / float(np.mean(tot)), 1)
        out["shape"] = f"{a.inflight} x {a.calls_per_pass}"
        print(json.dumps(out))
    finally:
        for c in ctxs:
            c.close()


if __name__ == "__main__":
    main()
