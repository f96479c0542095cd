#!/usr/bin/env python3
"""Fp Montgomery-product latency / throughput probe on cuda:0 (dependent chains)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

with GpuContext(0) as g:
    res = {"mad_peak_TMADs": g.mad_peak()[0] / 1e12}
    for lanes, iters in ((64, 2000), (256 * 64, 2000), (256 * 4 * 64, 1000), (256 * 16 * 64, 500),
                         (256 * 32 * 64, 500)):
        ns, rate = g.fpm_bench(lanes, iters)
        res[f"lanes={lanes}"] = {"ns_per_fpm_per_lane": round(ns, 1), "Gfpm_per_s": round(rate / 1e9, 3),
                                 "TMAD_per_s": round(rate * 288 / 1e12, 3)}
    print(json.dumps(res, indent=1))
