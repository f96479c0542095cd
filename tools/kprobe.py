#!/usr/bin/env python3
"""Latency probes (bls_gpu_kernel_probe) on cuda:0: one dependent 28-bit Fp product on a
lone lane (fpm_d28: 256 in a row), and [s] P on G1 by GLV with the window table in LDS
(glv_g1: k_pset's second wavefront, two lanes)."""
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

with GpuContext(0) as g:
    reps = 5
    out = {"fpm_d28_us_per_product_1_lane": round(g.kernel_probe("fpm_d28", 1, reps) / reps / 256 * 1e3, 4),
           "fpm_d28_us_per_product_64_lanes": round(g.kernel_probe("fpm_d28", 64, reps) / reps / 256 * 1e3, 4),
           "glv_g1_ms_2_lanes": round(g.kernel_probe("glv_g1", 2, reps) / reps, 4)}
    print(json.dumps(out))
