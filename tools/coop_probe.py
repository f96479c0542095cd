#!/usr/bin/env python3
"""Time the cooperative programs on cuda:0: us per step at 1 / 64 / 1024 tasks, and
per-step s_memtime stamps of one run split by step kind (product steps vs
linear-combination steps)."""
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
sys.path.insert(0, str(Path(__file__).resolve().parent))
import gen_coop  # noqa: E402
from lodestar_amd.native import GpuContext  # noqa: E402

progs, _ = gen_coop.build_all()
kinds = {p.name: [any(op.kind == 1 for op in st) for st in p.steps] for p in progs}
with GpuContext(0) as g:
    out = {}
    names = sys.argv[1:] or ["fin_fmul:200", "pset3_dbl_all:100", "pset3_add_1111:100", "pset3_phase2:3",
                             "pset3_ml2:3", "fin_fe2:2"]
    for item in names:
        name, reps = item.split(":")[0], int(item.split(":")[1])
        for blocks in (1, 1024, 3072):
            us, ms = g.coop_probe(name, blocks, reps)
            out[f"{name}@{blocks}"] = {"us_per_step": round(us, 3), "ms_per_run": round(ms / reps, 3)}
        k = np.array(kinds[name])
        _, _, st = g.coop_probe(name, 1, 1, 2 * len(k) + 1)
        st = st.astype(np.int64)  # s_memtime: shader-clock cycles; 2 stamps per step
        start, comp = st[0:-1:2], st[1::2]
        total = np.diff(st[0::2])
        compute = comp - start
        out[f"{name}:stamps"] = {
            "mul_steps": int(k.sum()), "mul_total": float(total[k].mean()) if k.any() else 0,
            "mul_compute": float(compute[k].mean()) if k.any() else 0,
            "lin_steps": int((~k).sum()), "lin_total": float(total[~k].mean()) if (~k).any() else 0,
            "lin_compute": float(compute[~k].mean()) if (~k).any() else 0}
    print(json.dumps(out, indent=1))
