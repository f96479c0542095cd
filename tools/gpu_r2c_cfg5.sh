#!/bin/bash
# cfg5 shape (2 signing roots per call, Miller-loop units) with k_mln4s vs the 380-slot
# k_mln<4>, then the calls-per-pass knee for cfg2 with k_mln4s.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/cfg5c
mkdir -p $O; cd $R
for rep in 1 2; do
  for v in 1 0; do
    BLS_ML_SMALL_FRAME=$v timeout -k 10 300 python -u bench.py --roots 2 --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/cfg5_${v}_$rep.json 2> $O/cfg5_${v}_$rep.err || { echo "cfg5 failed"; tail -5 $O/cfg5_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/cfg5_${v}_$rep.json'));print('cfg5 small=$v', round(d['value']), d['ms_per_step'])"
  done
done
for c in 3 5 6; do
  timeout -k 10 300 python -u bench.py --calls-per-pass $c --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/knee_8x$c.json 2> $O/knee_8x$c.err || { echo "knee failed"; tail -5 $O/knee_8x$c.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/knee_8x$c.json'));print('8x$c', round(d['value']), d['ms_per_step'])"
done
