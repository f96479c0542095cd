#!/usr/bin/env python3
"""Time the cooperative programs on cuda:0: us per step at 1 / 1024 tasks, and the
per-step s_memtime stamps of one run (step start, compute done): how much of a step
is the lanes' compute (operand gathers, product) and how much the write-back and the
wave sync.  Program names as in lodestar_amd/_native/coop_programs.json.

    python tools/coop_probe.py [name:reps ...]
"""
import json
import os
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

ROOT = Path(__file__).resolve().parent.parent
progs = json.loads((ROOT / "lodestar_amd" / "_native" / "coop_programs.json").read_text())
with GpuContext(0) as g:
    out = {}
    names = sys.argv[1:] or ["pset_dbl_all:100", "pset_add_x:100", "pset_phase2:3", "pset_ml2:3", "fin_fe2:2", "fin_fe1:2",
                             "pset_prep:3"]
    for item in names:
        name, reps = item.split(":")[0], int(item.split(":")[1])
        n_steps = progs[name]["steps"]
        for blocks in (1, 1024):
            us, ms = g.coop_probe(name, blocks, reps)
            out[f"{name}@{blocks}"] = {"us_per_step": round(us, 3), "ms_per_run": round(ms / reps, 3)}
        _, _, st = g.coop_probe(name, 1, 1, 2 * n_steps + 1)
        st = st.astype(np.int64)  # s_memtime (100 MHz constant clock on gfx9): 2 stamps per step
        start, comp = st[0:-1:2], st[1::2]
        total = np.diff(st[0::2])
        compute = comp - start
        out[f"{name}:stamps"] = {"steps": n_steps, "mul_steps": progs[name]["mul_steps"],
                                 "total_ticks_mean": float(total.mean()), "compute_ticks_mean": float(compute.mean()),
                                 "total_ticks_p10_p50_p90": [float(np.percentile(total, q)) for q in (10, 50, 90)]}
        # where a product step's time goes: ticks from step start to each stamp point
        # (coop.hpp coop_step, $BLS_COOP_PROBE_MARK), over the steps that reach point 3
        # (product steps, lane 0 a product)
        parts = {}
        for mark in (1, 2, 3, 4, 0):
            os.environ["BLS_COOP_PROBE_MARK"] = str(mark)
            _, _, sm = g.coop_probe(name, 1, 1, 2 * n_steps + 1)
            parts[mark] = sm.astype(np.int64)
        os.environ.pop("BLS_COOP_PROBE_MARK", None)
        mul = parts[3][1::2] != 0
        if mul.any():
            pts = {}
            for mark, label in ((1, "decoded"), (2, "operand_a"), (3, "operand_b"), (4, "product"), (0, "compute_done")):
                sm = parts[mark]
                d = (sm[1::2] - sm[0:-1:2])[mul]
                pts[label] = float(np.median(d))
            pts["step_total"] = float(np.median(np.diff(parts[0][0::2])[mul]))
            out[f"{name}:product_step_ticks_median"] = {"steps": int(mul.sum()), **pts}
    print(json.dumps(out, indent=1))
