#!/bin/bash
# k_mln packing (BLS_ML_PACK 4 vs 2): parity with the aggregated path forced on, then
# the cfg2 line for each packing (gpurun_out/mlpack)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/mlpack
mkdir -p $O
cd $R
BLS_SIGAGG=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_forced.log 2>&1 || { echo "pytest (forced) failed"; grep -E "FAIL|Error|assert" $O/pytest_forced.log | tail -30; exit 1; }
echo "forced: $(tail -1 $O/pytest_forced.log)"
for p in ${PACKS:-4 2}; do
  BLS_ML_PACK=$p timeout -k 10 300 python -u bench.py --steps 16 --warmup 4 --latency-runs 4 --no-cpu-baseline > $O/bench_$p.json 2> $O/bench_$p.err || { echo "bench failed"; tail -20 $O/bench_$p.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$p.json'));print('pack $p', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['stage_ms'])"
done
