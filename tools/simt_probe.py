"""Probe: throughput of the single-lane (one set per lane) exact path, k_exact, when
every set of a cfg2 call is forced through it (BLS_DEBUG_FORCE_EXACT), solo and with
several calls in flight.  Prints one JSON line per configuration."""
from __future__ import annotations

import json
import os
import sys
import threading
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))
os.environ.setdefault("GPU_MAX_HW_QUEUES", "24")

import bench  # noqa: E402
from lodestar_amd.native import GpuContext  # noqa: E402


def main():
    sets = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
    inflight = [int(x) for x in (sys.argv[2] if len(sys.argv) > 2 else "1,4,16").split(",")]
    ctxs = [GpuContext(0) for _ in range(max(inflight))]
    works = [bench.make_workload(c, sets, 0)[0] for c in ctxs]
    for c in ctxs:
        c.set_debug_flags(1)
    v, st = ctxs[0].verify_packed(works[0])
    assert (v == 1).all()
    for nf in inflight:
        reps = 2
        def run(i):
            for _ in range(reps):
                v, st = ctxs[i].verify_packed(works[i])
                assert (v == 1).all()
        th = [threading.Thread(target=run, args=(i,)) for i in range(nf)]
        t0 = time.perf_counter()
        for t in th:
            t.start()
        for t in th:
            t.join()
        dt = time.perf_counter() - t0
        _, st = ctxs[0].verify_packed(works[0])
        print(json.dumps({"sets": sets, "inflight": nf, "sets_per_s": round(sets * nf * reps / dt),
                          "stage_ms": [round(x, 3) for x in st.stage_ms], "flagged": st.n_flagged}), flush=True)
    for c in ctxs:
        c.close()


if __name__ == "__main__":
    main()
