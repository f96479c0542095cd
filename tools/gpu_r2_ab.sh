#!/bin/bash
# A/B of one environment switch on the cfg2 line, interleaved runs (gpurun_out/ab):
# $AB_VAR (e.g. BLS_GSUM_TREE), $AB_VALUES ("1 0"), $AB_REPS (2)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/ab
mkdir -p $O; cd $R
for rep in $(seq 1 ${AB_REPS:-2}); do
  for v in ${AB_VALUES:-1 0}; do
    tag=${AB_VAR}_${v}_$rep
    env $AB_VAR=$v timeout -k 10 300 python -u bench.py --steps 12 --warmup 3 --latency-runs 2 --no-cpu-baseline $BENCH_ARGS > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -5 $O/$tag.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'])"
  done
done
