#!/usr/bin/env python3
"""Throughput of the verifier with k concurrent in-flight batches (one context and
stream per host thread) on cuda:0."""
import json
import sys
import threading
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
from lodestar_amd.native import GpuContext  # noqa: E402

res = {}
ctxs = [GpuContext(0) for _ in range(4)]
work = [bench.make_workload(c, 1024, 0)[0] for c in ctxs]
for c, b in zip(ctxs, work):
    c.verify_packed(b)
for k in (1, 2, 3, 4):
    steps = 8
    def run(i):
        for _ in range(steps):
            v, _ = ctxs[i].verify_packed(work[i])
            assert (v == 1).all()
    ths = [threading.Thread(target=run, args=(i,)) for i in range(k)]
    t0 = time.perf_counter()
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    dt = time.perf_counter() - t0
    res[k] = {"sets_per_s": round(k * steps * 1024 / dt), "ms_per_batch": round(dt / (k * steps) * 1e3, 3)}
print(json.dumps(res))
