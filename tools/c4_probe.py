"""The cfg4 per-set-request slice's steady state with and without the range-sync slice run
on the same contexts before it (bench.py sub_records runs cfg4_slice first): wall rate
and per-pass device time of the failing passes, to tell a device slowdown from a host one.
Measurement tool, not part of the product.

  python tools/c4_probe.py [--before]"""
import argparse
import json
import os
import sys
import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def cpu_stat() -> dict:
    """the cgroup's CPU throttling counters (cgroup v2 cpu.stat), {} where absent"""
    try:
        return {k: int(v) for k, v in (ln.split() for ln in open("/sys/fs/cgroup/cpu.stat"))}
    except OSError:
        return {}


def steady(ctxs, w, cpp, jobs):
    from lodestar_amd import workloads as W

    pbs = W.packed_calls(w)
    bench.run_calls(ctxs, pbs[: len(ctxs) * cpp], cpp)
    c0, th0 = os.times(), cpu_stat()
    el, out, tot = bench.run_calls(ctxs, pbs * jobs, cpp)
    c1, th1 = os.times(), cpu_stat()
    npass = max(1, tot["passes"])
    return {"sets_per_s": round(jobs * w.n_sets / el, 1), "passes": tot["passes"],
            "cpu_s_per_wall_s": round((c1.user + c1.system - c0.user - c0.system) / el, 2),
            "cgroup_throttled": {k: th1.get(k, 0) - th0.get(k, 0) for k in ("nr_throttled", "throttled_usec")},
            "fail_device_ms_mean": round(tot["fail_device_ms"] / max(1, tot["merged_fail"] + tot.get("merged_skipped", 0)), 3),
            "pass_device_ms_sum_per_pass": round((tot["fail_device_ms"] + tot["pass_device_ms"]) / npass, 3),
            "wall_ms_per_pass_per_context": round(el * 1e3 / (npass / len(ctxs)), 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--contexts", type=int, default=16)
    ap.add_argument("--jobs", type=int, default=5)
    a = ap.parse_args()
    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    ctxs = [GpuContext(0) for _ in range(a.contexts)]
    res = {}
    try:
        W.load_table(ctxs, 1 << 20)
        wb = W.cfg4_slice(ctxs[0], 1 << 20, 125_000, batchable_calls=True)
        wr = W.cfg4_slice(ctxs[0], 1 << 20, 125_000, batchable_calls=False)
        c8 = ctxs[:8]
        res["batchable_first"] = steady(c8, wb, 64, a.jobs)
        res["range_sync"] = steady(c8, wr, 64, a.jobs)
        res["batchable_after_range_sync"] = steady(c8, wb, 64, a.jobs)
        res["batchable_again"] = steady(c8, wb, 64, a.jobs)
    finally:
        for c in ctxs:
            c.close()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
