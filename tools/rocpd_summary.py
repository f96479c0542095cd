#!/usr/bin/env python3
"""Per-kernel summary (calls, total / average / min / max duration) from a rocprofv3
rocpd database (rocprofv3 --kernel-trace --stats writes <name>_results.db).

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db > profiles/rNN_kernel_stats.csv
"""
import sqlite3
import sys

db = sqlite3.connect(sys.argv[1])
rows = db.execute(
    """select s.kernel_name, count(*), sum(d.end - d.start), avg(d.end - d.start), min(d.end - d.start),
              max(d.end - d.start), max(s.arch_vgpr_count), max(s.accum_vgpr_count), max(s.private_segment_size)
       from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id
       group by s.kernel_name order by sum(d.end - d.start) desc""").fetchall()
total = sum(r[2] for r in rows) or 1
print("Name,Calls,TotalDurationNs,AverageNs,MinNs,MaxNs,Percentage,ArchVGPR,AccumVGPR,ScratchBytesPerLane")
for name, calls, tot, avg, mn, mx, vg, ag, scr in rows:
    print(f"\"{name}\",{calls},{tot},{avg:.1f},{mn},{mx},{100.0 * tot / total:.2f},{vg},{ag},{scr}")
