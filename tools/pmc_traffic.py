"""Per-launch HBM traffic per kernel from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE), corrected as /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3)
prescribes for gfx950: FETCH_SIZE counts half the bytes of wide reads (x2),
WRITE_SIZE is exact; both are reported in KiB.

    python tools/pmc_traffic.py <fetch counter csv> <write counter csv> <out.json>

bench.py reads the newest profiles/*_pmc_traffic.json for roofline.traffic.
"""
from __future__ import annotations

import collections
import csv
import json
import sys


def per_launch(path: str, counter: str) -> dict:
    acc = collections.defaultdict(list)
    for row in csv.DictReader(open(path)):
        if row["Counter_Name"] == counter:
            name = row["Kernel_Name"].split("(")[0].split("<")[0].replace("void ", "").strip()
            acc[name].append(float(row["Counter_Value"]) * 1024.0)
    return {k: (sum(v) / len(v), len(v)) for k, v in acc.items()}


def main() -> None:
    fetch = per_launch(sys.argv[1], "FETCH_SIZE")
    write = per_launch(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        f, nf = fetch.get(k, (0.0, 0))
        w, nw = write.get(k, (0.0, 0))
        out[k] = {"fetch_bytes": 2.0 * f, "write_bytes": w, "hbm_bytes_per_launch": 2.0 * f + w,
                  "launches": [nf, nw], "correction": "FETCH_SIZE x2 (gfx950 wide-read undercount), KiB -> B"}
    json.dump(out, open(sys.argv[3], "w"), indent=1)
    print(json.dumps({k: round(v["hbm_bytes_per_launch"] / 1e6, 3) for k, v in out.items()}))


if __name__ == "__main__":
    main()
