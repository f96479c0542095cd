#!/bin/bash
# Interpreter operand prefetch (coop_lin) + 2-wave cap: GPU parity on the new build,
# then cfg2 (8 x 4) new vs previous build interleaved, p50@128, and the N-API line.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/pf
mkdir -p $O; cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 100 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
PREV=$R/lodestar_amd/_native/liblodestar_bls_prev.so
for rep in 1 2; do
  for v in new prev; do
    if [ $v = prev ]; then export LODESTAR_BLS_LIB=$PREV; else unset LODESTAR_BLS_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 2 --latency-runs 10 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench $v failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'], d['stage_ms'])"
  done
done
unset LODESTAR_BLS_LIB
timeout -k 10 400 python -u bench.py --mode napi --steps 30 --warmup 1 > $O/napi.json 2> $O/napi.err || { echo "napi failed"; tail -20 $O/napi.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/napi.json'));print('napi', round(d['value']), json.dumps(d['napi'])[:700])"
