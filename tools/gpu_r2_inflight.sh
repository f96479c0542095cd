#!/bin/bash
# cfg2 throughput vs calls in flight and HIP hardware queues (gpurun_out/inflight):
# $QUEUES (GPU_MAX_HW_QUEUES values), $INFLIGHT, $SIGAGG (BLS_SIGAGG values, "d" = default)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/inflight
mkdir -p $O
cd $R
for q in ${QUEUES:-4 16 32}; do
for m in ${SIGAGG:-d}; do
  for f in ${INFLIGHT:-16 32}; do
    tag=${q}_${m}_${f}
    if [ "$m" = d ]; then unset BLS_SIGAGG; else export BLS_SIGAGG=$m; fi
    GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --steps 8 --warmup 2 --inflight $f --latency-runs 2 --no-cpu-baseline > $O/b_$tag.json 2> $O/b_$tag.err || { echo "bench failed $tag"; tail -20 $O/b_$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/b_$tag.json'));print('queues $q sigagg $m inflight $f', round(d['value']), d['ms_per_step'])"
  done
done
done
