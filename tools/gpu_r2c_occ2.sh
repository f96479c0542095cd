#!/bin/bash
# k_mln4s A/B (cfg2, bench.py --steps 20): the default build vs the 380-slot k_mln<4>
# ($BLS_ML_SMALL_FRAME=0).  (Round 2c also ran a 2-waves/SIMD build of k_mln4s:
# profiles/r02c_ab_mln4s.json.)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/occ2
mkdir -p $O; cd $R
for rep in 1 2; do
  for v in w3 off; do
    case $v in
      w3) E="BLS_ML_SMALL_FRAME=1";;
      off) E="BLS_ML_SMALL_FRAME=0";;
    esac
    env $E timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 4 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['roofline']['frac'])"
  done
done
