#!/bin/bash
# In-flight knee for cfg2 with the final kernels: contexts x calls per pass, two reps.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/knee4
mkdir -p $O; cd $R
for rep in 1 2; do
  for cfg in 8x8 8x10 10x8 12x8; do
    i=${cfg%x*}; c=${cfg#*x}
    timeout -k 10 300 python -u bench.py --inflight $i --calls-per-pass $c --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/knee_${cfg}_$rep.json 2> $O/knee_${cfg}_$rep.err || { echo "knee $cfg failed"; tail -5 $O/knee_${cfg}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/knee_${cfg}_$rep.json'));print('$cfg', round(d['value']), d['ms_per_step'])"
  done
done
