#!/bin/bash
# The default bench line (with its cfg3 / cfg4 / cfg5 sub-records) under two environments
# in one call: ENVS="a:VAR=v,...;b:" (labels and variables as in gpu_r4.sh).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${TAG:-r5bab}; mkdir -p $O
for ab in $(echo "${ENVS:-base:}" | tr ';' ' '); do
  label=${ab%%:*}; vars=$(echo "${ab#*:}" | tr ',' ' ')
  env $vars timeout -k 10 700 python -u bench.py ${BENCH_ARGS} > $O/bench_$label.json 2> $O/bench_$label.err || { echo "bench $label failed"; tail -20 $O/bench_$label.err; exit 1; }
  python3 -c "
import json;d=json.load(open('$O/bench_$label.json'))
print('$label', d['value'], d['ms_per_step'], d.get('p50_latency_ms_128'), {k:(d[k].get('sets_per_s'),d[k].get('steady_sets_per_s')) for k in d if k.startswith(('cfg4','cfg5'))})"
done
