#!/usr/bin/env python3
"""Time the cooperative programs on cuda:0 (interpreter cost per step)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

with GpuContext(0) as g:
    out = {}
    for name, reps in (("fin_fmul", 200), ("fin_g2add", 100), ("fin_ml_neg_g1", 3), ("fin_fe2", 2)):
        for blocks in (1, 64, 1024):
            us, ms = g.coop_probe(name, blocks, reps)
            out[f"{name}@{blocks}"] = {"us_per_step": round(us, 3), "ms_per_run": round(ms / reps, 3)}
    print(json.dumps(out, indent=1))
