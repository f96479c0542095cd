#!/bin/bash
# In-flight knee for cfg2 with k_mln4s: contexts x calls per pass.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/knee3
mkdir -p $O; cd $R
for cfg in 8x8 8x10 10x6 12x4 16x4 6x8; do
  i=${cfg%x*}; c=${cfg#*x}
  timeout -k 10 300 python -u bench.py --inflight $i --calls-per-pass $c --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/knee_$cfg.json 2> $O/knee_$cfg.err || { echo "knee $cfg failed"; tail -5 $O/knee_$cfg.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/knee_$cfg.json'));print('$cfg', round(d['value']), d['ms_per_step'])"
done
