#!/bin/bash
# kernel trace of the default bench (gpurun_out/trace), then one stream's sequence
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/trace
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --latency-runs 2 --steps 6 --warmup 1 $BENCH_ARGS > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cd $R
f=$(find $O/t -name "*kernel_trace.csv" | head -1)
python3 tools/trace_timeline.py $f k_mln | tail -1
python3 - "$f" <<'PY'
import csv, sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if r['Kind']=='KERNEL_DISPATCH']
qs=sorted(set(r['Queue_Id'] for r in rows), key=lambda q: -sum(1 for r in rows if r['Queue_Id']==q))
q=qs[3]
rs=sorted([r for r in rows if r['Queue_Id']==q], key=lambda r:int(r['Start_Timestamp']))
idx=[i for i,r in enumerate(rs) if r['Kernel_Name'].startswith('k_pk')]
i0=idx[len(idx)//2]
t0=int(rs[i0]['Start_Timestamp']); prev=None
for r in rs[i0:i0+16]:
    s=int(r['Start_Timestamp']); e=int(r['End_Timestamp'])
    print(f"{(s-t0)/1e6:8.3f} +{((s-prev)/1e6 if prev else 0):6.3f} {(e-s)/1e6:7.3f} {r['Kernel_Name'][:40]}")
    prev=e
PY
