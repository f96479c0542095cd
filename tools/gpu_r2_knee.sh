#!/bin/bash
# Where cfg2 throughput saturates (contexts x calls per pass), then the N-API path with
# the same coalescing (gpurun_out/knee).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/knee
mkdir -p $O; cd $R
for cfg in ${KNEE_CFGS:-"8 4" "8 6" "10 4" "12 4" "16 4" "8 8"}; do
  set -- $cfg
  tag=i$1_k$2
  timeout -k 10 300 python -u bench.py --inflight $1 --calls-per-pass $2 --steps ${STEPS:-10} --warmup 2 --latency-runs 2 --no-cpu-baseline > $O/$tag.json 2> $O/$tag.err || { echo "fail $tag"; tail -5 $O/$tag.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/$tag.json'));print('$tag', round(d['value']), d['ms_per_step'])"
done
timeout -k 10 400 python -u bench.py --mode napi --steps 30 --warmup 1 > $O/napi.json 2> $O/napi.err || { echo "napi failed"; tail -20 $O/napi.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/napi.json'));print('napi', round(d['value']), json.dumps(d['napi'])[:600])"
