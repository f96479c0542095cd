"""Latency probe: one 128-set call (cfg1 shape, bench.py's p50_latency_ms_128) or one
cfg2 call of N sets, repeated; prints the median wall time and the stage times the
library reports.  Run under `rocprofv3 --kernel-trace` for per-kernel durations.

    python tools/lat_probe.py [--sets 128] [--runs 10] [--batchable]
"""
import argparse
import json
import statistics
import sys
import time
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))

import bench  # noqa: E402
from lodestar_amd.native import GpuContext, pack_requests  # noqa: E402


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", type=int, default=128)
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--batchable", action="store_true", help="one batchable request per set (cfg2 shape)")
    ap.add_argument("--no-check", action="store_true", help="timing builds that skip work: verdicts not checked")
    args = ap.parse_args()
    gpu = GpuContext(0)
    _, _, sets, _ = bench.make_workload(gpu, max(args.sets, 128), 0)
    sets = sets[:args.sets]
    call = pack_requests([(True, [s]) for s in sets]) if args.batchable else pack_requests([(False, sets)])
    gpu.verify_packed(call)  # warm-up
    lat, stages = [], []
    for _ in range(args.runs):
        t = time.perf_counter()
        v, st = gpu.verify_packed(call)
        lat.append((time.perf_counter() - t) * 1e3)
        stages.append([round(x, 3) for x in st.stage_ms[:]])
        assert args.no_check or all(x == 1 for x in v)
    print(json.dumps({"sets": args.sets, "batchable": args.batchable, "p50_ms": round(statistics.median(lat), 3),
                      "stage_names": bench.STAGE_NAMES, "stage_ms_last": stages[-1]}))
    gpu.close()


if __name__ == "__main__":
    main()
