#!/bin/bash
# k_fprod skips exact ones (7 of 8 Miller-loop items of a shared loop): GPU parity
# suite, then the cfg2 and cfg5 bench lines at the 8 x 8 default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/skip1
mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
for rep in 1 2; do
  timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 4 --no-cpu-baseline > $O/bench_$rep.json 2> $O/bench_$rep.err || { echo "bench failed"; tail -5 $O/bench_$rep.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/bench_$rep.json'));print('cfg2', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['roofline']['frac'])"
done
timeout -k 10 300 python -u bench.py --roots 2 --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; tail -5 $O/cfg5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5', round(d['value']), d['ms_per_step'])"
