#!/bin/bash
# Final round-2 lines with the 8 x 8 default: the driver-shaped bench (with the CPU
# baseline), the N-API mode, and a kernel trace of the same bench command.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/final3
mkdir -p $O; cd $R
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
timeout -k 10 400 python -u bench.py --mode napi --steps 30 --warmup 1 > $O/bench_napi.json 2> $O/bench_napi.err || { echo "napi bench failed"; tail -20 $O/bench_napi.err; exit 1; }
cat $O/bench_napi.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --latency-runs 2 --steps 4 --warmup 1 > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
cd $R
python3 tools/trace_timeline.py $(find $O/trace -name "*kernel_trace.csv" | head -1) k_mln > $O/timeline.txt
tail -1 $O/timeline.txt
