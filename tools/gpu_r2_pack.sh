#!/bin/bash
# parity tests, then cfg2 bench with 2 and 3 sets per wavefront
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pack
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for P in 3 2; do
  BLS_PACK=$P timeout -k 10 300 python -u bench.py --steps 48 --warmup 2 --no-cpu-baseline --latency-runs 3 > $O/bench_p$P.json 2> $O/bench_p$P.err || { echo "bench P=$P failed"; tail -20 $O/bench_p$P.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_p$P.json'));print('P=$P', d['value'], d['p50_latency_ms_128'], d['stage_ms'], d['roofline']['work'])"
done
