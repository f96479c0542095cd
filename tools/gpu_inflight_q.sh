#!/bin/bash
# bench at several (in-flight batches, hardware queues) pairs, one line each
set -o pipefail
mkdir -p gpurun_out
for P in ${SWEEP:-12:16 16:16 16:24 20:24 24:24}; do
  B=${P%%:*}; Q=${P##*:}
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 200 python -u bench.py --no-cpu-baseline --inflight $B --steps 96 --latency-runs 3 > gpurun_out/bench_if${B}_q$Q.log 2>&1 || { echo "bench $P failed"; tail -20 gpurun_out/bench_if${B}_q$Q.log; exit 1; }
  python -c "import json; d=json.loads(open('gpurun_out/bench_if${B}_q$Q.log').read().strip().splitlines()[-1]); print('$P', d['value'], d['ms_per_step'])"
done
