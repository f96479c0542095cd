#!/bin/bash
# bench at several in-flight batch counts (one line each)
set -o pipefail
mkdir -p gpurun_out
for B in ${SWEEP:-2 3 4 6 8}; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --inflight $B --steps 24 --latency-runs 3 > gpurun_out/bench_if$B.log 2>&1 || { echo "bench $B failed"; tail -20 gpurun_out/bench_if$B.log; exit 1; }
  python -c "import json,sys; d=json.loads(open('gpurun_out/bench_if$B.log').read().strip().splitlines()[-1]); print($B, d['value'], d['ms_per_step'], d['stage_ms'])"
done
