"""Knee of the cfg4 per-GPU slice (range-sync replay: 128-set calls, 10 % aggregates of
128 keys, 1 % invalid) against the sets in flight: contexts x calls per pass, both call
shapes (non-batchable calls and per-set batchable requests), verdicts checked.  Writes
one JSON object to stdout; bench.py's cfg4 sub-record defaults come from it.

  python tools/sweep_cfg4.py [--sets 125000] [--grid 4x32,8x32,12x32,8x64,12x64]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main() -> None:
    import bench
    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=125_000)
    ap.add_argument("--keys", type=int, default=1 << 20)
    ap.add_argument("--grid", default="4x32,8x32,12x32,8x64,12x64")
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    grid = [tuple(int(x) for x in g.split("x")) for g in a.grid.split(",")]
    n_ctx = max(c for c, _ in grid)
    ctxs = [GpuContext(0) for _ in range(n_ctx)]
    out = {"sets": a.sets, "points": []}
    try:
        W.load_table(ctxs, a.keys)
        for batchable in (False, True):
            w = W.cfg4_slice(ctxs[0], a.keys, a.sets, batchable_calls=batchable)
            pbs = W.packed_calls(w)
            for c, cpp in grid:
                bench.run_calls(ctxs[:c], pbs[: c * cpp], cpp)  # warm-up
                best = None
                for _ in range(a.reps):
                    el, res, _ = bench.run_calls(ctxs[:c], pbs, cpp)
                    best = el if best is None else min(best, el)
                    bad = [k for k in range(len(pbs)) if not W.verdicts_ok(w, k, res[k])]
                    assert not bad, f"{len(bad)} wrong verdicts"
                pt = {"batchable": batchable, "contexts": c, "calls_per_pass": cpp, "sets_in_flight": c * cpp * 128,
                      "elapsed_s": round(best, 4), "sets_per_s": round(w.n_sets / best, 1)}
                out["points"].append(pt)
                print(json.dumps(pt), file=sys.stderr, flush=True)
    finally:
        for x in ctxs:
            x.close()
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    t0 = time.time()
    main()
    print(f"[sweep_cfg4] {time.time() - t0:.1f} s", file=sys.stderr)
