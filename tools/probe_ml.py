#!/usr/bin/env python3
"""Design probe on cuda:0: Miller-loop pairs/s of the cooperative shared 8-pair program
(ml1s_8, the verify path's k_mlns<8>) against one SIMT Miller loop per lane
(kernels/k_probe.hip ml_simt_*), and the 28-bit-digit product rate by occupancy.
Writes one JSON object to stdout."""
import json
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from lodestar_amd.native import GpuContext  # noqa: E402

res = {}
with GpuContext(0) as g:
    res["mad_peak_TMADs"] = round(g.mad_peak()[0] / 1e12, 3)
    for waves in (1, 2, 4, 8):
        lanes = 64 * 1024 * waves
        ms = g.kernel_probe("fpm_d28", lanes, 3)
        res[f"fpm_d28_{waves}w_per_simd"] = {"Gfpm_per_s": round(3 * lanes * 256 / (ms * 1e-3) / 1e9, 2)}
    for name in ("ml_simt_w1", "ml_simt_w2"):
        for waves in (1, 2):
            lanes = 64 * 1024 * waves
            t0 = time.time()
            ms = g.kernel_probe(name, lanes, 2)
            res[f"{name}_{lanes}_lanes"] = {"ms_per_launch": round(ms / 2, 3),
                                            "pairs_per_s": round(2 * lanes / (ms * 1e-3)), "wall_s": round(time.time() - t0, 2)}
    for blocks in (256 * 6, 256 * 12):
        us, ms = g.coop_probe("ml1s_8", blocks, 3)
        res[f"ml1s_8_{blocks}_blocks"] = {"ms_per_launch": round(ms / 3, 3), "pairs_per_s": round(3 * blocks * 8 / (ms * 1e-3))}
print(json.dumps(res))
