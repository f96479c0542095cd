"""bench.py's sub-records alone (cfg3 / cfg4_slice / cfg4_slice_batchable / cfg5_slice /
cfg5_slice_valid), for A/B runs of the failing-pass paths under environment knobs:

  python tools/sub_probe.py --only cfg4_slice_batchable,cfg5_slice [--jobs 5] [--reps 2]

prints one JSON object {record: {...}} with the same fields as the default line's
records (sets/s of one job, steady_sets_per_s of back-to-back jobs, verdicts checked)."""
import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402  (sets GPU_MAX_HW_QUEUES before the library loads)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="cfg4_slice_batchable,cfg5_slice")
    ap.add_argument("--table-keys", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--jobs", type=int, default=5)
    ap.add_argument("--detail", action="store_true", help="per-pass device times of each --only slice instead")
    ap.add_argument("--contexts", type=int, default=12, help="contexts opened (cfg5 runs on all; cfg4 on --cfg4-contexts)")
    ap.add_argument("--cfg4-contexts", type=int, default=12)
    ap.add_argument("--cfg4-calls-per-pass", type=int, default=64)
    a = ap.parse_args()
    if a.detail:
        print(json.dumps({k: detail(k) for k in a.only.split(",")}))
        return
    res = bench.sub_records(a.table_keys, a.contexts, 22, 125_000, reps=a.reps, cfg4_ctx=a.cfg4_contexts,
                            cfg4_cpp=a.cfg4_calls_per_pass, jobs=a.jobs,
                            only=set(a.only.split(",")))
    res["env"] = {k: v for k, v in os.environ.items() if k.startswith("BLS_")}
    print(json.dumps(res))



def detail(key: str, jobs: int = 2):
    """Per-pass device times of one slice's steady state: passes whose merged check
    failed against those that passed, and the failed passes' stages."""
    import numpy as np

    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    ctxs = [GpuContext(0) for _ in range(12)]
    try:
        W.load_table(ctxs, 1 << 20)
        if key.startswith("cfg4"):
            w = W.cfg4_slice(ctxs[0], 1 << 20, 125_000, batchable_calls=key.endswith("batchable"))
            c, cpp = ctxs[:8], 64
        else:
            w = W.cfg5_slice(ctxs[0], 1 << 20, 131_072, 256, invalid=64)
            c = ctxs
            cpp = (len(W.packed_calls(w)) + 11) // 12
        pbs = W.packed_calls(w)
        bench.run_calls(c, pbs[: len(c)], 1)
        el, out, tot = bench.run_calls(c, pbs * jobs, cpp)
        nf = max(1, tot["merged_fail"] + tot.get("merged_skipped", 0))
        npass = max(1, tot["passes"] - tot["merged_fail"] - tot.get("merged_skipped", 0))
        return {"sets_per_s": round(jobs * w.n_sets / el, 1), "passes": tot["passes"], "failed": tot["merged_fail"],
                "skipped": tot.get("merged_skipped", 0),
                "fail_device_ms_mean": round(tot["fail_device_ms"] / nf, 3),
                "pass_device_ms_mean": round(tot["pass_device_ms"] / npass, 3),
                "fail_stage_ms_mean": {k: round(float(x) / nf, 3) for k, x in zip(bench.STAGE_NAMES,
                                                                                   tot["fail_stage_ms"])},
                "fail_fallback_ms_mean": round((tot["fail_device_ms"] - float(np.sum(tot["fail_stage_ms"]))) / nf, 3)}
    finally:
        for x in ctxs:
            x.close()


if __name__ == "__main__":
    main()
