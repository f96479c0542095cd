#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3 4; do
timeout -k 10 200 python -u bench.py --steps 24 --warmup 2 --inflight $k --no-cpu-baseline --latency-runs 5 > gpurun_out/bench_if$k.log 2>&1 || { tail -5 gpurun_out/bench_if$k.log; exit 1; }
python -c "import json;d=json.loads(open('gpurun_out/bench_if$k.log').read().strip().splitlines()[-1]);print($k, d['value'], d['ms_per_step'], d['stage_ms'])"
done
