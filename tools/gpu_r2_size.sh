#!/bin/bash
# Throughput vs GPU-call size at a fixed number of sets in flight (gpurun_out/size):
# the same cfg2 sets coalesced into fewer, larger verifyManySignatureSets calls.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/size
mkdir -p $O; cd $R
for cfg in ${SIZE_CFGS:-"1024 20" "2048 10" "2048 16" "4096 8" "1024 28"}; do
  set -- $cfg
  tag=s$1_i$2
  timeout -k 10 300 python -u bench.py --sets $1 --inflight $2 --steps ${STEPS:-12} --warmup 2 --latency-runs 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'], d['stage_ms'])"
done
