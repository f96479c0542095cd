#!/usr/bin/env python3
"""Concurrency of a rocprofv3 kernel trace (kernel_trace.csv): per kernel name the
dispatch count, mean duration, scratch and registers, and over the busiest window the
mean number of kernels and wavefronts resident at once, with the queue ids in use.

    python tools/trace_timeline.py <kernel_trace.csv> [kernel substring to window on]
"""
import collections
import csv
import sys


def main() -> None:
    rows = list(csv.DictReader(open(sys.argv[1])))
    key = sys.argv[2] if len(sys.argv) > 2 else "k_mln"
    ks = [r for r in rows if r["Kind"] == "KERNEL_DISPATCH"]
    for r in ks:
        r["t0"], r["t1"] = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        r["waves"] = (int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"])) // 64
    per = collections.defaultdict(list)
    for r in ks:
        per[r["Kernel_Name"].split("(")[0]].append(r)
    for name, rs in sorted(per.items(), key=lambda x: -sum(r["t1"] - r["t0"] for r in x[1])):
        d = [r["t1"] - r["t0"] for r in rs]
        r0 = rs[0]
        print(f"{name[:40]:40s} n={len(rs):4d} mean={sum(d) / len(d) / 1e6:8.3f} ms waves={r0['waves']:5d} "
              f"scratch={r0['Scratch_Size']} vgpr={r0['VGPR_Count']}+{r0['Accum_VGPR_Count']} lds={r0['LDS_Block_Size']}")
    sel = [r for r in ks if key in r["Kernel_Name"]]
    if not sel:
        return
    lo, hi = min(r["t0"] for r in sel), max(r["t1"] for r in sel)
    ev = []
    for r in ks:
        a, b = max(r["t0"], lo), min(r["t1"], hi)
        if a < b:
            ev.append((a, 1, r["waves"]))
            ev.append((b, -1, -r["waves"]))
    ev.sort()
    nk = nw = 0
    last = lo
    acc_k = acc_w = 0.0
    for t, dk, dw in ev:
        acc_k += nk * (t - last)
        acc_w += nw * (t - last)
        nk += dk
        nw += dw
        last = t
    span = hi - lo
    queues = collections.Counter(r["Queue_Id"] for r in ks if lo <= r["t0"] <= hi)
    print(f"window {span / 1e6:.1f} ms (first..last {key}): mean kernels in flight {acc_k / span:.2f}, "
          f"mean waves launched-and-unfinished {acc_w / span:.0f}, queues {dict(queues)}")


if __name__ == "__main__":
    main()
