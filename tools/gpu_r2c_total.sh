#!/bin/bash
# Merged signature sum ($BLS_SIG_TOTAL, bls_gpu.hip use_total): probe (valid call, one
# invalid set -> per-chunk re-sum), GPU parity suite, then cfg2 / cfg5 A/B at 8 x 8.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/total
mkdir -p $O; cd $R
BLS_DEBUG_SYNC=1 timeout -k 10 90 python -u tools/sigagg_probe.py 1024 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -E "k_mln|k_chunk|valid|invalid" $O/probe.log | head -8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  for v in 1 0; do
    BLS_SIG_TOTAL=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('total=$v', round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
  done
done
for v in 1 0; do
  BLS_SIG_TOTAL=$v timeout -k 10 300 python -u bench.py --roots 2 --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/cfg5_$v.json 2> $O/cfg5_$v.err || { echo "cfg5 failed"; tail -5 $O/cfg5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cfg5_$v.json'));print('cfg5 total=$v', round(d['value']), d['ms_per_step'])"
done
