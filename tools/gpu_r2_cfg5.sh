#!/bin/bash
# cfg5 shape (1024-set calls over 2 committee-shared roots): Miller-loop units on / off,
# dedup off (gpurun_out/cfg5)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cfg5
mkdir -p $O
cd $R
for v in "" "--no-units" "--no-dedup"; do
  tag=cfg5${v// /_}
  timeout -k 10 300 python -u bench.py --roots 2 --steps 16 --warmup 4 --latency-runs 2 --no-cpu-baseline $v > $O/$tag.json 2> $O/$tag.err || { echo "bench failed $tag"; tail -20 $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'], d['stage_ms'])"
done
