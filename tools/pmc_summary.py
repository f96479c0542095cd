#!/usr/bin/env python3
"""Condense rocprofv3 --pmc passes (one counter_collection.csv per pass) into the JSON
summary bench.py reads (profiles/r*_pmc_k_pset*.json).

    python tools/pmc_summary.py [--sets-per-pass N] [--shape TEXT] <out.json> <note> <pass dir>...

Per kernel (averaged over its dispatches): the raw counters, plus
  waves_per_simd   = SQ_WAVE_CYCLES x 4 / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs): resident
                     wavefronts per SIMD over the dispatch (SQ_WAVE_CYCLES counts
                     quad-cycles; GRBM_GUI_ACTIVE sums the 8 XCDs, MI355X_MICROARCH.md);
  valu_busy        = SQ_ACTIVE_INST_VALU x 4 / (GRBM_GUI_ACTIVE / 8 x 1024): the share of
                     SIMD cycles issuing a VALU instruction;
  clock_ghz        = GRBM_GUI_ACTIVE / 8 / dispatch time (when a kernel trace is given);
  hbm_bytes_per_launch = FETCH_SIZE x 2 + WRITE_SIZE (KiB -> B; gfx950 counts half the
                     bytes of wide reads, the guide's correction).
With --sets-per-pass: sets_per_pass, shape and per_dispatch_valu_wave_insts_per_set
(SQ_INSTS_VALU of every dispatch / sets per pass, in dispatch order; bench.py takes each
kernel's minimum as the timed pass shape).
"""
from __future__ import annotations

import collections
import csv
import glob
import json
import sys


def load(pass_dir: str) -> dict:
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{pass_dir}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"].split("(")[0].replace("void ", "").strip()
            acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return acc


def main() -> None:
    argv = sys.argv[1:]
    sets_per_pass, shape = None, None
    while argv and argv[0].startswith("--"):
        if argv[0] == "--sets-per-pass":
            sets_per_pass = int(argv[1])
        elif argv[0] == "--shape":
            shape = argv[1]
        argv = argv[2:]
    out_path, note, dirs = argv[0], argv[1], argv[2:]
    merged = collections.defaultdict(dict)
    for d in dirs:
        for name, ctrs in load(d).items():
            for c, v in ctrs.items():
                merged[name][c] = sum(v) / len(v)
    kernels = {}
    for name, c in merged.items():
        k = dict(c)
        cyc = c.get("GRBM_GUI_ACTIVE", 0) / 8.0
        if cyc and "SQ_WAVE_CYCLES" in c:
            k["waves_per_simd"] = round(c["SQ_WAVE_CYCLES"] * 4 / (cyc * 1024), 3)
        if cyc and "SQ_ACTIVE_INST_VALU" in c:
            k["valu_busy"] = round(c["SQ_ACTIVE_INST_VALU"] * 4 / (cyc * 1024), 3)
        if "FETCH_SIZE" in c or "WRITE_SIZE" in c:
            k["hbm_bytes_per_launch"] = int((2.0 * c.get("FETCH_SIZE", 0) + c.get("WRITE_SIZE", 0)) * 1024)
        k["note"] = note
        kernels[name] = k
    out = {"source": "rocprofv3 --pmc, one pass per counter group: " + " ".join(dirs), "kernels": kernels}
    if sets_per_pass:
        per = {}
        for d in dirs:
            for name, ctrs in load(d).items():
                if "SQ_INSTS_VALU" in ctrs:
                    per[name] = [round(v / sets_per_pass) for v in ctrs["SQ_INSTS_VALU"]]
        out.update({"sets_per_pass": sets_per_pass, "shape": shape or note, "per_dispatch_valu_wave_insts_per_set": per})
    json.dump(out, open(out_path, "w"), indent=1)
    for name, k in kernels.items():
        if any(t in name for t in ("pset", "k_mln", "k_chain", "k_pre", "k_mlq", "k_mlf", "k_msm", "k_fprod")):
            ipw = round(k["SQ_INSTS_VALU"] / k["SQ_WAVES"]) if k.get("SQ_WAVES") and "SQ_INSTS_VALU" in k else None
            print(name, {x: k.get(x) for x in ("waves_per_simd", "valu_busy", "hbm_bytes_per_launch", "SQ_WAVES")},
                  "valu_insts_per_wave", ipw)


if __name__ == "__main__":
    main()
