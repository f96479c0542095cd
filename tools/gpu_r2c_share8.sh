#!/bin/bash
# k_mlns<8> ($BLS_ML_SHARE=8: eight sets of a chunk share one 8-pair Miller loop) at
# the 8 x 8 bench default: GPU parity suite under it, then cfg2 / cfg5 A/B against
# k_mlns<4>.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/share8
mkdir -p $O; cd $R
BLS_ML_SHARE=8 BLS_DEBUG_SYNC=1 timeout -k 10 90 python -u tools/sigagg_probe.py 1024 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -E "k_mln|valid|invalid" $O/probe.log | head -6
BLS_ML_SHARE=8 timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  for v in 8 4; do
    BLS_ML_SHARE=$v timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('share=$v', round(d['value']), d['ms_per_step'], d['roofline']['frac'])"
  done
done
for v in 8 4; do
  BLS_ML_SHARE=$v timeout -k 10 300 python -u bench.py --roots 2 --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/cfg5_$v.json 2> $O/cfg5_$v.err || { echo "cfg5 failed"; tail -5 $O/cfg5_$v.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/cfg5_$v.json'));print('cfg5 share=$v', round(d['value']), d['ms_per_step'])"
done
