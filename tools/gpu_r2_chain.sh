#!/bin/bash
# k_chain + k_mln ($BLS_CHAIN=1) and k_chain + k_mls ($BLS_CHAIN=2) vs the
# all-cooperative k_pset: parity, the cfg2 bench line for each, kernel traces
# (gpurun_out/chain).  $MODES: the BLS_CHAIN values to bench (default "1 2").
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/chain
mkdir -p $O
cd $R
export TMPDIR=/tmp
MODES=${MODES:-"1 2"}
for m in $MODES; do
  BLS_CHAIN=$m timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu_$m.log 2>&1 || { echo "pytest failed ($m)"; grep -E "FAIL|Error|assert" $O/pytest_gpu_$m.log | tail -30; exit 1; }
  echo "mode $m: $(tail -1 $O/pytest_gpu_$m.log)"
  BLS_CHAIN=$m timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline > $O/bench_$m.json 2> $O/bench_$m.err || { echo "bench failed"; tail -20 $O/bench_$m.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$m.json'));print('mode $m', d['value'], d['p50_latency_ms_128'], d['stage_ms'])"
  BLS_CHAIN=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_$m -o chain -- python3 bench.py --steps 4 --warmup 1 --no-cpu-baseline > $O/prof_$m.log 2>&1 || { echo "rocprof failed"; tail -20 $O/prof_$m.log; exit 1; }
  f=$(find $O/prof_$m -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_$m.csv
  python3 - <<PY
import csv
for r in csv.DictReader(open("$O/kernel_stats_$m.csv")):
    print("  ", r["Name"][:50], r["Calls"], r["AverageNs"], r["Percentage"])
PY
done
