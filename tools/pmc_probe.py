#!/usr/bin/env python3
"""Run one cooperative program (argv[1], default pset_ml2) on 1024 tasks for PMC
collection under rocprofv3 --pmc (one program per kernel dispatch of k_coop_probe)."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "pset_ml2"
with GpuContext(0) as g:
    us, ms = g.coop_probe(name, 1024, 2)
    print(name, "us/step", round(us, 3), "ms", round(ms, 3))
