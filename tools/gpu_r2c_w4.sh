#!/bin/bash
# k_chain roles 2-3 ([r] sig, [r] pk) with a fixed 4-bit window instead of
# double-and-add: probe, GPU parity suite, then cfg2 / cfg5 A/B against the build
# variant chain_binr (double-and-add) at the 8 x 8 default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/w4
mkdir -p $O; cd $R
BLS_DEBUG_SYNC=1 timeout -k 10 90 python -u tools/sigagg_probe.py 1024 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -E "k_chain|valid|invalid" $O/probe.log | head -6
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; grep -E "FAIL|Timeout|Error|assert" $O/pytest_gpu.log | tail -30; exit 1; }
tail -1 $O/pytest_gpu.log
B=$R/lodestar_amd/_native/liblodestar_bls_chain_binr.so
for rep in 1 2; do
  for v in w4 binr; do
    if [ $v = binr ]; then export LODESTAR_BLS_LIB=$B; else unset LODESTAR_BLS_LIB; fi
    timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/bench_${v}_$rep.json 2> $O/bench_${v}_$rep.err || { echo "bench failed"; tail -5 $O/bench_${v}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/bench_${v}_$rep.json'));print('$v', round(d['value']), d['ms_per_step'], d['p50_latency_ms_128'])"
  done
done
unset LODESTAR_BLS_LIB
timeout -k 10 300 python -u bench.py --roots 2 --steps 20 --warmup 5 --latency-runs 2 --no-cpu-baseline > $O/cfg5.json 2> $O/cfg5.err || { echo "cfg5 failed"; tail -5 $O/cfg5.err; exit 1; }
python3 -c "import json;d=json.load(open('$O/cfg5.json'));print('cfg5 w4', round(d['value']), d['ms_per_step'])"
