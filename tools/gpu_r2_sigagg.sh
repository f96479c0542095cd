#!/bin/bash
# aggregated-signature path: parity with the path forced on ($BLS_SIGAGG=1) and by
# size (default), the cfg2 bench line, a kernel trace (gpurun_out/sigagg)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/sigagg
mkdir -p $O
cd $R
export TMPDIR=/tmp
BLS_SIGAGG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_forced.log 2>&1 || { echo "pytest (forced) failed"; grep -E "FAIL|Error|assert" $O/pytest_forced.log | tail -30; exit 1; }
echo "forced: $(tail -1 $O/pytest_forced.log)"
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_default.log 2>&1 || { echo "pytest (default) failed"; grep -E "FAIL|Error|assert" $O/pytest_default.log | tail -30; exit 1; }
echo "default: $(tail -1 $O/pytest_default.log)"
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/bench.json'));print('cfg2', d['value'], d['p50_latency_ms_128'], d['roofline']['frac'], d['stage_ms'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o sigagg -- python3 bench.py --steps 4 --warmup 1 --latency-runs 2 --no-cpu-baseline > $O/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - <<PY
import csv
for r in csv.DictReader(open("$O/kernel_stats.csv")):
    print("  ", r["Name"][:50], r["Calls"], r["AverageNs"], r["Percentage"])
PY
python3 tools/trace_timeline.py $O/prof/sigagg_kernel_trace.csv k_mln
