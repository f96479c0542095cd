"""One cfg3 block-import call (bench.py sub-record cfg3: 128 aggregate sets x 512 keys + a
512-key sync aggregate over a 1M-key device table), repeated, for a kernel trace of its
stages.  Prints p50 and the summed per-stage device times.

  python tools/cfg3_probe.py [--runs 10] [--table-keys 1048576]
"""
import argparse
import json
import os
import statistics
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=10)
    ap.add_argument("--table-keys", type=int, default=1 << 20)
    args = ap.parse_args()
    from lodestar_amd import workloads as W
    from lodestar_amd.native import GpuContext

    with GpuContext(0) as gpu:
        W.load_table([gpu], args.table_keys)
        w = W.cfg3_block(gpu, args.table_keys)
        pb = W.packed_calls(w)[0]
        gpu.verify_packed(pb)  # warm-up
        lat, stage = [], np.zeros(8)
        for _ in range(args.runs):
            t0 = time.perf_counter()
            v, st = gpu.verify_packed(pb)
            lat.append(time.perf_counter() - t0)
            stage += np.array(st.stage_ms[:])
            assert W.verdicts_ok(w, 0, v)
    print(json.dumps({"sets": w.n_sets, "p50_ms": round(statistics.median(lat) * 1e3, 3),
                      "stage_names": ["h2d", "k_pk", "k_pre", "k_chain", "sig_sums", "miller_loops",
                                      "k_status+k_chunk", "k_indiv"],
                      "stage_ms_mean": [round(float(x) / args.runs, 3) for x in stage]}))


if __name__ == "__main__":
    main()
